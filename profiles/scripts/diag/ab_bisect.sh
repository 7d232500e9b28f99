for n in d1 y0 g0 all0; do echo "== $n"; VIHMC_LIB=$GRAFT_REPO_ROOT/_var/$n.so timeout -k 10 100 python profiles/scripts/diag/contract_ab.py 1 16 || exit 1; done
