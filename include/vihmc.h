/*
 * vihmc.h -- C-ABI of libvihmc.so, the MI355X (gfx950) log-posterior + gradient engine for VI-HMC.
 *
 * It replaces the reference's log-probability closure: the Python callable returned by
 * `define_model_log_prob` and handed to hamiltorch's sampler.
 *   - DeepONet VI-HMC:  Operator_network/VI_HMC/main_VI_HMC_burgers.py:27-180
 *                       (log_prob_func :86-178, Functional_DeepONet my_make_func.py:44-83)
 *   - DeepONet full HMC / splitting shards: Operator_network/HMC/main_HMC_splitting.py:79-258
 *   - BNN VI-HMC:       Neural_network/VI_HMC/main_VI_HMC.py:28-153 (Functional_Net my_make_func.py:52-73)
 *   - BNN full HMC:     hamiltorch.define_model_log_prob as called by
 *                       Neural_network/HMC/main_regression_hmc.py:124-127 (same function, 'regression' loss)
 * and the forward used by `predict_model` (main_VI_HMC_burgers.py:183-241, main_VI_HMC.py:156-259).
 *
 * Where the reference evaluates ONE parameter vector per call through PyTorch autograd, a plan here
 * evaluates C chains at once: theta is [C, K] (K = number of sampled / "sensitive" parameters),
 * logp is [C] and grad is [C, K]. All three are DEVICE pointers on the plan's device; inputs given
 * at plan creation are HOST pointers and are copied (the plan owns its device copies).
 *
 * Conventions
 *   - every function returns 0 on success, a nonzero code on failure; vihmc_last_error() gives a
 *     thread-local message. A non-finite log-probability is NOT an error: it is returned as is and
 *     the caller treats it as a rejection (reference: util.LogProbError, util.py:107-119).
 *   - `stream` is a hipStream_t passed as void* (0 = the null stream). Calls only enqueue work;
 *     there is no host synchronisation inside vihmc_logp_grad / vihmc_forward.
 *   - results are deterministic: fixed-order reductions, no floating-point atomics.
 *   - a plan is bound to one device and used from one host thread.
 */
#ifndef VIHMC_H
#define VIHMC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vihmc_plan vihmc_plan;

enum vihmc_act  { VIHMC_ACT_IDENTITY = 0, VIHMC_ACT_TANH = 1, VIHMC_ACT_RELU = 2, VIHMC_ACT_SINE = 3 };
enum vihmc_loss { VIHMC_LOSS_NLL = 0,       /* GaussianNLLLoss(sum), tau_out = variance  (:83-84,162-163) */
                  VIHMC_LOSS_REGRESSION = 1 /* -0.5*tau_out*sum(r^2), tau_out = precision (:157-159)     */ };

/* One nn.Linear: weight[n_out, n_in] at w_off and bias[n_out] at b_off (-1: no bias) in the flat
 * parameter vector (util.unflatten order, Operator_network/VI_HMC/util.py:141-152). `act` is the
 * activation applied to this layer's output (VIHMC_ACT_IDENTITY for the last layer of each MLP). */
typedef struct {
    int64_t w_off, b_off;
    int32_t n_out, n_in, act, _pad;
} vihmc_linear;

/* Gaussian log-likelihood + Gaussian prior shared by both model kinds. */
typedef struct {
    int32_t loss;          /* enum vihmc_loss                                                     */
    float   tau_out;       /* variance (NLL) or precision (regression)                            */
    float   prior_scale;   /* prior divided by this (splitting shards: num_splits, :253-254)      */
    int32_t _pad;
} vihmc_lik_desc;

/* DeepONet: `branch` and `trunk` are the layer tables of DeepONet's b1 / b2 Sequentials
 * (Operator_network/VI_HMC/model.py:42-62); the scalar output bias b sits at flat index 0.
 * Trunk inputs are given already mapped to features (my_make_func.py:63-65, theta-independent). */
typedef struct {
    int32_t n_branch_layers, n_trunk_layers;
    const vihmc_linear* branch;
    const vihmc_linear* trunk;
    int64_t n_params;      /* D                                   */
    int32_t N;             /* branch rows (functions)             */
    int32_t P;             /* trunk rows (space-time points)      */
    int32_t in_branch;     /* branch input width                  */
    int32_t in_trunk;      /* trunk feature width                 */
    int32_t K;             /* sampled parameters per chain        */
    int32_t max_chains;    /* largest C ever passed to this plan  */
    vihmc_lik_desc lik;
} vihmc_deeponet_desc;

/* BNN MLP (Neural_network/VI_HMC/main_VI_HMC.py:297-334): layers in Sequential order. */
typedef struct {
    int32_t n_layers;
    int32_t _pad0;
    const vihmc_linear* layers;
    int64_t n_params;      /* D                       */
    int32_t N;             /* data rows               */
    int32_t in_dim;        /* input width             */
    int32_t out_dim;       /* output width            */
    int32_t K;
    int32_t max_chains;
    int32_t _pad1;
    vihmc_lik_desc lik;
} vihmc_mlp_desc;

/* Create a DeepONet plan.
 *   x_branch [N, in_branch] fp32, trunk_feat [P, in_trunk] fp32, y [N, P] fp32,
 *   frozen [D] fp32: the weights that are not sampled (mu_VI; `sampled_weights` at my_make_func.py:21,48),
 *   sens_idx [K] int64: sorted indices of the sampled parameters (gradient_indices_*.npy); K == D with
 *            sens_idx = 0..D-1 is full-parameter HMC (mus=None branch, my_make_func.py:45-46),
 *   prior_mu [K], prior_sd [K] fp32: Normal(prior_mu, prior_sd) per sampled parameter (:74-81,96-102).
 * Replaces: define_model_log_prob(...) (main_VI_HMC_burgers.py:27-84), incl. the torch.load of mu/sigma. */
int vihmc_deeponet_plan_create(vihmc_plan** out, const vihmc_deeponet_desc* d,
                               const float* x_branch, const float* trunk_feat, const float* y,
                               const float* frozen, const int64_t* sens_idx,
                               const float* prior_mu, const float* prior_sd, int device);

/* Create a BNN plan (x [N, in_dim], y [N, out_dim]). Replaces Neural_network/VI_HMC/main_VI_HMC.py:28-95;
 * prior_mu/prior_sd already expanded per sampled parameter with the reference's per-tensor slicing
 * (main_VI_HMC.py:107-112). */
int vihmc_mlp_plan_create(vihmc_plan** out, const vihmc_mlp_desc* d,
                          const float* x, const float* y,
                          const float* frozen, const int64_t* sens_idx,
                          const float* prior_mu, const float* prior_sd, int device);

/* log p(theta_c) and d log p / d theta_c for C <= max_chains chains.
 * Replaces: log_prob_func(params) + torch.autograd.grad(log_prob, params) [hamiltorch params_grad],
 * main_VI_HMC_burgers.py:86-178 / main_VI_HMC.py:96-151. grad may be NULL (value only). */
int vihmc_logp_grad(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, void* stream);

/* d log p / d theta_c only (no log-prob): the leapfrog's inner gradient evaluations (hamiltorch's params_grad
 * between the position updates, SURVEY.md App. A.2, whose log-prob value is discarded). DeepONet plans with
 * width 100 and max_chains >= the plan option "gram_min_chains" use the Gram-form contraction (vihmc_gram.hip: no N x P
 * residual, plan option "gram"); vihmc_trajectory uses the same path for its inner steps. */
int vihmc_grad(vihmc_plan* p, const float* theta, int C, float* grad, void* stream);

/* One HMC iteration's Metropolis step for C chains of K parameters, all device pointers, one launch. Replaces the
 * accept block of hamiltorch's sample loop (samplers.py: H0 = -lp0 + ke0, H1 = -lp1 + ke1 from the caller's kinetic
 * energies [C] of the opening / closing momenta, rho = min(H0 - H1, 0) with NaN -> 0, a chain whose log-prob is not
 * finite fails (hamiltorch's LogProbError: no accept), accept = rho >= logu[c]), batched as
 * vihmc.samplers.HMCRunner.step does it: after burn-in (burn = 0) an accepted proposal (th1, lp1, g1) overwrites
 * the last returned state in place and, when samples != NULL, the state is written to row counts[c] of
 * samples [C][s_cap][K] (a failed chain's row to row s_cap - 1, uncounted) and counts[c] advances; rows 0 .. s_cap - 2
 * hold samples: once counts[c] reaches s_cap - 1 further states go to the spare row uncounted; during burn-in
 * (burn = 1) th_cur / lp_cur / g_cur receive the proposal, else (failed) the last returned state, else the
 * fallback th_bp / lp_bp / g_bp, which an accepted proposal replaces. accepted[c * acc_ld + n], trace[c * tr_ld + n]
 * (the state's log-prob), rho [C] (NaN where failed) and err [C] are written. */
int vihmc_hmc_accept(int C, int K, int n, int burn, const float* lp0, const float* lp1, const float* ke0,
                     const float* ke1, const float* logu, const float* th1, const float* g1,
                     float* th_last, float* lp_last, float* g_last, float* th_bp, float* lp_bp, float* g_bp,
                     float* th_cur, float* lp_cur, float* g_cur, float* samples, int64_t s_cap, int64_t* counts,
                     uint8_t* accepted, int64_t acc_ld, float* trace, int64_t tr_ld, float* rho, uint8_t* err,
                     void* stream);

/* Kinetic energies ke[c] = 0.5 sum_k p[c][k] inv_mass[k] p[c][k] (inv_mass [K] device or NULL = identity) of C
 * chains of K parameters, p [C][K] device, in ONE launch. Replaces hamiltorch's kinetic term of `hamiltonian`
 * (0.5 p.p, or 0.5 p.(inv_mass p)) that HMCRunner computed as 0.5 * (p * p).sum(1) -- four
 * launches. Summed in fp64 in a fixed order (slice partials, then the slices in order), rounded once to fp32.
 * Workspace: part [C * vihmc_kinetic_slices(K)] doubles and cnt [C] uint32 ZEROED before the first call (every call
 * leaves them zeroed again); one workspace per stream. */
int vihmc_kinetic_slices(int K);
int vihmc_kinetic(const float* p, const float* inv_mass, int C, int K, float* ke, double* part, uint32_t* cnt,
                  void* stream);

/* Forward only: logp [C] and the network output out [C, N, P] (DeepONet) or [C, N, out_dim] (BNN).
 * Replaces log_prob_func(..., predict=True) -> (logp, output) (main_VI_HMC_burgers.py:175-176). */
int vihmc_forward(vihmc_plan* p, const float* theta, int C, float* logp, float* out, void* stream);

/* BNN plans: one whole leapfrog trajectory of every chain in ONE launch (hamiltorch leapfrog,
 * Sampler.HMC with the implicit integrator): from theta_in [C, K], the fresh momentum
 * p_in [C, K] and the gradient g_in [C, K] at theta_in, L steps of size eps[c] (device [C]; inv_mass [K]
 * device or NULL) -> theta_out, p_out (after the final half-step), g_out and logp_out [C] at theta_out.
 * Every product and sum is rounded separately (no fused multiply-add), so the result is bitwise the step-by-
 * step path (L vihmc_logp_grad calls between the torch updates). Replaces hamiltorch's leapfrog loop over
 * params_grad for the BNN configs (Neural_network/{HMC,VI_HMC}); fails for DeepONet plans. */
int vihmc_mlp_trajectory(vihmc_plan* p, const float* theta_in, float* theta_out, const float* p_in, float* p_out,
                         const float* g_in, float* g_out, float* logp_out, const float* eps, const float* inv_mass,
                         int L, int C, void* stream);

/* Any plan: one whole leapfrog trajectory, the contract of vihmc_mlp_trajectory (which it calls for BNN plans).
 * DeepONet plans: one opening kernel (p = p_in + (eps/2) g_in; theta = theta_in + eps p) and L evaluations
 * whose gradient gather applies the momentum step and the next position step in place (theta_out and p_out
 * hold the running state; no torch elementwise kernels per step). Same rounding as the step-by-step path,
 * so the result is bitwise that path. Replaces hamiltorch's leapfrog loop over params_grad
 *  for every config's Sampler.HMC / HMC_NUTS trajectory. */
int vihmc_trajectory(vihmc_plan* p, const float* theta_in, float* theta_out, const float* p_in, float* p_out,
                     const float* g_in, float* g_out, float* logp_out, const float* eps, const float* inv_mass,
                     int L, int C, void* stream);

/* DeepONet plans: one gradient evaluation of a data shard inside hamiltorch's Integrator.SPLITTING trajectory over
 * two shards with the end gradient reused (Operator_network/HMC/main_HMC_splitting.py:361-369, config 4; the
 * momentum / position updates of HMCRunner._trajectory around that evaluation), the updates
 * applied in place by the evaluation's gradient gather instead of torch elementwise kernels:
 *   mode 1: p += kick g; p += kick g; theta += drift p   (this shard's two kicks, then the drift to the next shard)
 *   mode 2: p += kick g                                  (the trajectory's last kick)
 * each update one fma, as torch.add(x, y, alpha=a), so the trajectory is bitwise the torch-op path. theta [C, K]
 * and p [C, K] are device arrays updated in place (theta is also this evaluation's input). grad [C, K] receives g;
 * logp [C] (or NULL: gradient only) the log-prob at the input theta. scatter_into (mode 1, may be NULL): the plan
 * of the NEXT evaluation (same network layout), into whose packed weights / images the gather writes the new
 * theta, which that evaluation then skips with scattered_in = 1. */
int vihmc_split_step(vihmc_plan* p, float* theta, float* momentum, int C, float* grad, float* logp, int mode, float kick,
                     float drift, vihmc_plan* scatter_into, int scattered_in, void* stream);

/* Plan introspection: 0 = DeepONet, 1 = MLP; D; K; max_chains; device bytes owned. */
/* Sensitivity scores of every parameter at theta (chain 0 of the plan, [K] device):
 *   out[d] = sigma[d]^2 * mean over outputs of (d f / d theta_d)^2,  d < D, flat (named_parameters) order.
 * DeepONet: the outputs are f[n][pts[n][k]], n < N, k < npts; pts is HOST memory [N][npts] int32 (the
 *   trunk points each validation function samples, BurgersDataSet.__getitem__ at
 *   Operator_network/VI/utils.py:39-41). BNN: every data row and output; pts ignored.
 * sigma [D] device or NULL (then out = the mean squared gradient). out [D] device.
 * Replaces eval_std_dydw + eval_jac (Operator_network/VI/sensitivity.py:62-126,
 * Neural_network/VI/sensitivity.py:71-126; torch.func.jacrev over all D parameters). Synchronises
 * `stream` before returning (temporaries are freed). */
int vihmc_sensitivity(vihmc_plan* p, const float* theta, const int32_t* pts, int npts, const float* sigma,
                      float* out, void* stream);

/* Replace the data of a DeepONet plan (same N and P): x_branch [N, in_branch] and y [N, P], device
 * pointers, copied into the plan on `stream` (ordered before later evaluations on it). For minibatch loops
 * (Operator_network/VI/main_VI_deeponet.py:58-79) without re-creating the plan. */
int vihmc_plan_set_data(vihmc_plan* p, const float* x_branch, const float* y, void* stream);

/* cfg.sample_data (Operator_network/VI_HMC/main_VI_HMC_burgers.py:131-134, `ind = sample(range(x2.shape[1]),
 * cfg.p)`): make the plan's P trunk rows the rows ind[0..P) of the full grid. trunk_all [P_all, in_trunk]
 * (trunk features), y_all [N, P_all], ind [P] int32 in [0, P_all) -- all device pointers; the caller draws and
 * checks the indices. Gathered on `stream` (ordered before later evaluations on it); a pure copy. */
int vihmc_plan_set_trunk_rows(vihmc_plan* p, const float* trunk_all, const float* y_all, int64_t P_all,
                              const int32_t* ind, void* stream);

int     vihmc_plan_kind(const vihmc_plan* p);
int64_t vihmc_plan_n_params(const vihmc_plan* p);
int     vihmc_plan_K(const vihmc_plan* p);
int     vihmc_plan_max_chains(const vihmc_plan* p);
int64_t vihmc_plan_device_bytes(const vihmc_plan* p);

/* Kernel-level timing hook for the roofline: when a class is enabled, HIP events bracket every launch of
 * that kernel class on the evaluation's stream. vihmc_timing_enable(p, which, on) turns class `which` (or all
 * classes, which = -1) on / off and discards recorded events; vihmc_timing_read_class sums the recorded
 * launches of one class (-1: all) without discarding them (it syncs their events); vihmc_timing_read sums all
 * and discards; vihmc_timing_reset discards. The evaluation is not captured into a hipGraph while timing. */
enum {
    VIHMC_T_CONTRACT_A = 0,   /* side-A contraction: S, Gaussian NLL, G, dZ_trunk (k_contract_bf / k_contract_ws) */
    VIHMC_T_CONTRACT_B = 1,   /* side-B contraction: dZ_branch = G Z_trunk (k_contract_bf_b / k_contract2) */
    VIHMC_T_BWD = 2,          /* layer backward, one launch per layer (k_bwd_bf / k_bwd_ws); one event pair brackets
                                 the consecutive layer launches and counts them all (boundaries included) */
    VIHMC_T_FWD = 3,          /* fused hidden-layer forward (k_fwd_fused_bf / k_fwd_fused) */
    VIHMC_T_EVAL = 4,         /* one whole DeepONet evaluation, first to last launch */
    VIHMC_T_MLP = 5,          /* BNN evaluation (k_mlp) */
    VIHMC_T_GRAM = 6,         /* Gram-form gradient-only contraction (k_gram_aug, k_gram_a, k_gram_b): one
                                 event pair brackets the four launches */
    VIHMC_T_COUNT = 7
};
int vihmc_timing_enable(vihmc_plan* p, int which, int on);
int vihmc_timing_read(vihmc_plan* p, double* total_ms, int64_t* launches);
int vihmc_timing_read_class(vihmc_plan* p, int which, double* total_ms, int64_t* launches);
int vihmc_timing_reset(vihmc_plan* p);

/* hipGraph replay of vihmc_logp_grad (gradient evaluations only): one graph per chain count, captured
 * on first use, over plan-owned theta/logp/grad buffers that the call copies in / out on `stream`.
 * Off by default (measured slightly slower than direct launches here); the VIHMC_GRAPH=1 environment
 * variable turns it on for every plan. (New; no reference counterpart.) */
int vihmc_graph_enable(vihmc_plan* p, int on);

/* Plan options (new; no reference counterpart): "fwd_bf16x6" (default 1) computes the hidden 100->100
 * layers of the forward with every fp32 product split exactly into three bf16 parts on the bf16 MFMA
 * (six products, fp32 accumulation: fp32-level results, ~4 % faster evaluation); 0 = fp32 MFMA.
 * "contract_bf16x6" (default 1): the same for the side-A contraction (branch x trunk S, likelihood,
 * G, dZ_trunk; width 100) and side B. "bwd_bf16x6" (default 1): the same for the layer backward (dX,
 * dW, db of layers with 100 outputs); its default (environment VIHMC_BWD_BF16) also sizes the backward
 * row chunks at plan creation. "graph" = vihmc_graph_enable. "gram" (default 1): gradient-only DeepONet
 * evaluations (vihmc_grad, the inner steps of vihmc_trajectory) in Gram form; "gram_min_chains" (default 4): the
 * smallest plan max_chains that uses it (default 4: below it the residual form's split sweeps fill the chip better;
 * decided per plan, so a chain's trajectory does not depend on the call's chain count). "grad_evals" / "gram_evals"
 * (read: gradient-evaluation calls since creation / of which in Gram form; set: any value resets both; direct
 * launches only). Changing an option drops captured graphs.
 * Returns nonzero for an unknown key. */
int vihmc_plan_option(vihmc_plan* p, const char* key, int value);
/* Current value of an option (contract_bf16x6 reads 1 only where the bf16x6 contraction applies,
 * i.e. width 100; graph reads -1 while it follows VIHMC_GRAPH). */
int vihmc_plan_get_option(const vihmc_plan* p, const char* key, int* value);

/* Bounds audit (new; no reference counterpart): a plan created with the environment variable VIHMC_CANARY=1 gives
 * every device buffer it owns a 4-KB tail of 0xA5 bytes that no kernel may write. This synchronises the device and
 * returns in *corrupted the number of tail bytes that changed (0 = no out-of-bounds write into a plan buffer); it
 * fails for plans created without the variable. */
int vihmc_plan_check_canaries(vihmc_plan* p, int64_t* corrupted);

/* Diagnostics (new; no reference counterpart): synchronise the device and copy the named internal buffer of a
 * DeepONet plan (all max_chains chains) into host memory dst; dst == NULL only returns its size in *bytes (0: not
 * allocated). Names: dzb, dzt, act_b, act_t, bimg, timg, gram_tb, gram_tb_sum, gram_gt_part, gram_gb_part, gram_gt,
 * gram_gb, gram_tt, gram_stats. */
int vihmc_plan_debug_copy(vihmc_plan* p, const char* name, void* dst, int64_t* bytes);

/* Measurement (new; no reference counterpart): enqueue on `stream` one stamp of the shader clock. out is DEVICE
 * memory [256][4] uint64: per one-wave workgroup its XCD id, HW_ID register (CU / shader array / engine),
 * s_memtime (shader-clock ticks) and s_memrealtime (100 MHz ticks). Two stamps around a timed region give each CU's
 * average shader clock over it from that CU's own two readings: (d memtime / d memrealtime) x 100 MHz (bench.py:
 * "sclk_mhz", medians per XCD). */
int vihmc_clock_stamp(uint64_t* out, void* stream);

void        vihmc_plan_destroy(vihmc_plan* p);
const char* vihmc_last_error(void);
/* "vihmc <ver> gfx950 diag=<n>": the VIHMC_DIAG value (csrc/vihmc_diag.h: timing-only ablations and phase stamps) the
 * library was built with (0 in a product build). Plan creation fails in a build with VIHMC_DIAG != 0 unless
 * VIHMC_ALLOW_DIAG=1 (A/B timing of variant builds only: results are wrong by design). */
const char* vihmc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VIHMC_H */
