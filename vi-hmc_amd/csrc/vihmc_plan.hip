// Plan management and the extern "C" boundary of libvihmc.so (declared in include/vihmc.h).
//
// A DeepONet plan owns, per chain c < max_chains:
//   packed weights  [dp]   : b0 slot, then per layer  Wp[n_out][ldi] | bias[n_out] | WT[n_in][ldo]
//                            (ld* = round_up(.,4) so every row is 16-B aligned for float4 operand loads;
//                            padding stays zero), initialised once from the frozen vector (mu_VI);
//                            each evaluation only scatters theta into the K sampled positions.
//   activations     per net: h_j [rows][ldo_j] for every layer j (needed by the backward)
//   deltas          per net: 2 ping-pong buffers [rows][max ldo]
//   gradient        [dp]   : packed layout (Wp | bias) + slot 0 for db0, gathered at the sampled indices
//   partial slabs   side-B contraction partials and per-row-chunk dW/db partials (fixed-order reduce)
// Shared across chains: branch input [N][ldxb], trunk features [P][ldxt], y [N][P] and y^T [P][N].
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "vihmc.h"
#include "vihmc_internal.h"
#include <cstdlib>
#include <cstdio>

using namespace vihmc;

namespace {

thread_local std::string g_err;
constexpr size_t CANARY_BYTES = 4096;

int fail(const std::string& msg, int code = 1) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) return fail(std::string(#expr) + ": " + hipGetErrorString(e_), (int)e_); \
    } while (0)

inline int64_t r4(int64_t x) { return (x + 3) & ~int64_t(3); }
inline int64_t r64(int64_t x) { return (x + 63) & ~int64_t(63); }
inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

struct LayerPk {
    int n_out, n_in, ldi, ldo, act;
    int64_t wp, bias, wt;
    // dW partials: one slab per row chunk of rows_per_chunk rows
    int n_chunks, rows_per_chunk;
    int64_t part_off, part_stride;
};

struct Net {
    std::vector<LayerPk> L;
    int rows = 0, ld_in = 0;
    float* input = nullptr;       // shared [rows][ld_in]
    float* act = nullptr;         // per chain
    int64_t act_cs = 0;
    std::vector<int64_t> h_off;
    float* delta[2] = {nullptr, nullptr};
    int64_t delta_cs = 0;
    float* dwpart = nullptr;
    int64_t dwpart_cs = 0;
    int rows_per_chunk = 256;
};

}  // namespace

struct vihmc_plan {
    int kind = 0;  // 0 DeepONet, 1 MLP
    int device = 0;
    int64_t D = 0;
    int K = 0, maxC = 0;
    vihmc_lik_desc lik{};
    std::vector<void*> allocs;
    int64_t bytes = 0;
    // bounds audit (environment VIHMC_CANARY=1 at plan creation): every plan buffer gets a CANARY_BYTES tail of
    // 0xA5 that no kernel may write; vihmc_plan_check_canaries counts the tail bytes that changed
    bool canary = [] {
        const char* e = std::getenv("VIHMC_CANARY");
        return e && std::atoi(e) != 0;
    }();
    std::vector<unsigned char*> canaries;
    // bounds audit of reads too (environment VIHMC_GUARD=1 at plan creation): every buffer is placed at the end of its
    // own HIP virtual-memory mapping, followed by an unmapped granule, so an access more than 255 B past its end
    // faults at once instead of landing in a neighbouring allocation (debug runs only: each buffer takes whole granules)
    bool guard_pages = [] {
        const char* e = std::getenv("VIHMC_GUARD");
        return e && std::atoi(e) != 0;
    }();
    struct VmmBuf {
        void* base;
        size_t total, mapped;
        hipMemGenericAllocationHandle_t h;
    };
    std::vector<VmmBuf> vmm;
    hipError_t vmm_alloc(void** out, size_t sz) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t g = 0;
        e = hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum);
        if (e != hipSuccess) return e;
        const size_t m = (sz + g - 1) / g * g, total = m + g;
        VmmBuf b{nullptr, total, m, {}};
        if ((e = hipMemAddressReserve(&b.base, total, 0, nullptr, 0)) != hipSuccess) return e;
        if ((e = hipMemCreate(&b.h, m, &prop, 0)) != hipSuccess) return e;
        if ((e = hipMemMap(b.base, m, 0, b.h, 0)) != hipSuccess) return e;
        hipMemAccessDesc ad{};
        ad.location = prop.location;
        ad.flags = hipMemAccessFlagsProtReadWrite;
        if ((e = hipMemSetAccess(b.base, m, &ad, 1)) != hipSuccess) return e;
        vmm.push_back(b);
        *out = static_cast<unsigned char*>(b.base) + (m - (sz + 255) / 256 * 256);
        // VIHMC_GUARD_POISON=k: the bytes of allocation k (-1: every allocation) behind its end, up to the guard, read
        // as NaN (0xFF) -- a kernel that uses them poisons its result (the alloc zeroes [ptr, ptr + sz) afterwards)
        const char* pe = std::getenv("VIHMC_GUARD_POISON");
        const int poison = pe ? std::atoi(pe) : -2;
        const int k = (int)vmm.size() - 1;
        if (poison == -1 || poison == k)
            if ((e = hipMemset(b.base, 0xFF, m)) != hipSuccess) return e;
        if (std::getenv("VIHMC_GUARD_VERBOSE")) fprintf(stderr, "vihmc guard alloc #%d: %zu bytes\n", k, sz);
        return hipSuccess;
    }

    int32_t* smap_w = nullptr;
    int32_t* smap_wt = nullptr;
    int32_t* smap_img = nullptr;    // per sampled index: byte offset of its weight-image plane element, or -1
    int32_t* smap_imgf = nullptr;   // ... of its fp32 image copy (k tail / bias), or -1
    bool img_by_scatter = false;    // the weight images are split once and kept current by k_scatter
    float* prior_mu = nullptr;
    float* prior_iv = nullptr;
    double prior_const = 0.0;
    float* lik_buf = nullptr;
    double* lp_part = nullptr;            // [maxC][GATHER_SPLIT_MAX] partial log-priors
    uint32_t* fin_cnt = nullptr;          // [maxC] blocks of the gradient gather done (its last block finalises)

    // DeepONet
    int N = 0, P = 0, W = 0, ldz = 0;
    Net nets[2];
    float* packed = nullptr;
    float* gp = nullptr;
    int64_t dp = 0;
    float* y = nullptr;
    float* gT = nullptr;        // per chain G^T [P][ldgT] (side A -> side B); gT_cs floats per chain
    int64_t gT_cs = 0;
    int ldgT = 0;               // N rounded up to 32 floats: every row starts on a 128-B line; the bf16x6
                                // kernels use the same bytes chunk-blocked ([N/32][P][32])
    unsigned char* qsplitA = nullptr;   // per chain: branch outputs pre-split for k_contract_bf (W = 100)
    int64_t qsplitA_cs = 0;             // bytes per chain
    unsigned char* qsplitB = nullptr;   // per chain: trunk outputs pre-split for k_contract_bf_b
    int64_t qsplitB_cs = 0;
    bool img_by_fwd = false;            // this evaluation's fused forward wrote qsplitA / qsplitB
    float* partB = nullptr;
    int64_t partB_cs = 0;
    int qchunksB = 1, qperB = 32;
    int qchunksA = 1, qperA = 32;          // side A splits its q range only for small chain counts
    float* partA = nullptr;
    int64_t partA_cs = 0;
    ReduceJob* jobsA = nullptr;            // (qchunksA > 1) the side-B and side-A reduce jobs, one launch
    int lenA = 0;
    double* stats = nullptr;
    int64_t stats_cs = 0;
    int nwavesA = 0;
    ReduceJob* jobsB = nullptr;
    ReduceJob* jobsW = nullptr;      // dW partial reduces: row-major slabs (fp32 backward)
    ReduceJob* jobsWt = nullptr;     // ... tiled slabs for the layers the bf16x6 backward kernels run
    uint8_t* gsamp = nullptr;        // [dp] 1 at the packed positions of sampled parameters (K < D only)
    int n_jobsW = 0, max_lenW = 0, lenB = 0;
    int spanA = 0, spanB = 0, spanW = 0, spanWt = 0;   // k_reduce grid extents of the job lists (reduce_span)

    std::vector<int32_t> fmap_host;    // flat parameter index -> packed offset (sensitivity output map)

    // MLP
    MlpArgs mlp{};
    int maxw = 0;

    // timing hook: HIP events bracket every launch of the enabled kernel classes (vihmc.h VIHMC_T_*) on the
    // evaluation's stream; ev_cls[i] is the class of the event pair (2i, 2i+1)
    int timing_on = 0;              // bit mask of enabled classes
    int timing_every = 1;           // plan option: events on every n-th DeepONet evaluation only (bench sampling)
    int64_t n_evals = 0;            // DeepONet evaluations so far (timing_every's phase)
    std::vector<hipEvent_t> ev_pool;
    std::vector<int> ev_cls;       // class of pair i
    std::vector<int> ev_nl;        // launches the pair brackets (the layer backward: one pair around all layers)
    size_t ev_used = 0;

    // hipGraph replay of the gradient evaluation: one captured graph per chain count C, over plan-owned
    // theta / logp / grad buffers (the caller's tensors are copied in / out around the launch), so an
    // evaluation is 4 stream operations instead of ~20 kernel launches
    std::vector<std::pair<int, hipGraphExec_t>> graphs;
    hipStream_t cap_stream = nullptr;
    // bf16x6 forward: weights pre-split (kept current by the scatter, or k_split_wimg per evaluation) and
    // DMA-staged; plan option fwd_wimg = 0 runs the fp32-MFMA fused forward instead (the bf16x6 one reads the
    // images' fp32 k tail)
    unsigned char* wimg = nullptr;
    int64_t wimg_cs = 0;
    unsigned char* wtimg = nullptr;   // the backward's transposed images (BWD_WTIMG per fused layer), same upkeep
    int64_t wtimg_cs = 0;
    int32_t* smap_timg = nullptr;     // per sampled index: byte offset of its W^T-image plane element, or -1
    int32_t* smap_timgf = nullptr;    // ... of its fp32 n-tail copy, or -1
    int fwd_wimg = 1;
    int fwd_in0 = 1;              // plan option: the input layers inside the bf16x6 forward's launch (FusedNet::x)
    int skip_zt = 1;              // plan option: all-Gram evaluations store no fp32 copy of the trunk's outputs
    int fuse_scatter = 1;       // plan option: trajectory evaluations take theta already scattered by the leapfrog
    int mlp_fast = 1;             // plan option: the reference BNN shape on the register-resident kernels (vihmc_bnn.hip)
    int bwd_chain = 1;            // plan option: whole-network backward in one launch when the chunks are 64 rows
    // Gram-form gradient-only contraction (vihmc_gram.hip) for the evaluations that return no log-prob (the
    // trajectory's inner leapfrog steps, vihmc_grad): plan options "gram" (on / off) and "gram_min_chains"
    // (gradient-only evaluation, Gram vs residual form, ms: C = 2 0.40 vs 0.34, C = 4 0.50 vs 0.53, C = 16 1.36 vs 1.48;
    // profiles/r03x_gram_crossover.txt)
    int gram = 1, gram_min_chains = 4;
    bool gram_alloc = false;      // W = 100 plan: images and work buffers allocated
    __bf16* gya = nullptr;        // y [NG*256][32 nblkP], 3 planes (kpos order inside each 32-long p block)
    __bf16* gyb = nullptr;        // y^T [PT*256][32 nblkN], 3 planes
    int64_t gya_plane = 0, gyb_plane = 0;
    int gya_ld = 0, gyb_ld = 0, gNG = 0, gS = 0, gSL = 0, gPT = 0, gSB = 1, gSLB = 1, gSt = 1, gSLt = 1;
    int gStc = 1, gSLtc = 1;      // the centred form's Gram-t units (units of their own: any split, GRAM_T_SPLIT x S)
    float* gtt_part = nullptr;    // T_t split-K slabs (gSB > 1)
    int64_t gtt_cs = 0;
    float* gtb_part = nullptr;
    int64_t gtb_cs = 0;
    double* ggt_part = nullptr;
    int64_t ggt_part_cs = 0;
    int gSb = 1, gSLb = 1;        // Gram-b slabs (ggb_part) of gSLb branch blocks
    double* ggb_part = nullptr;
    int64_t ggb_part_cs = 0;
    float* gtb_sum = nullptr;     // summed T_b slabs (gS > GRAM_TB_DIRECT)
    int64_t gtbs_cs = 0;
    float* ggt = nullptr;
    double* ggt64 = nullptr;      // [C][112][112] Gt in fp64 (the dZb epilogue)
    unsigned char* ggb = nullptr;
    unsigned char* ggb3 = nullptr;  // [C][4 blocks][32][112] bf16: the 4th plane of -Gb (k_gram_b extension blocks)
    double* gstats = nullptr;
    int64_t gstats_cs = 0;
    // Centred data (plan option gram_center, default 1; round 6): the Gram form runs on y~ = y - S0, S0 =
    // B0 T0^T + b0 the network output at the centre weights (the frozen vector, chain 0's packed weights at creation),
    // so its two data products scale with the residual, not with y. Built lazily (ensure_centre) before the first
    // evaluation that needs it after creation / a data change, on chain 0's slot with its state saved around it.
    int gram_center = 1;
    int gram_pair2 = 0;               // plan option: centred T_t units of two chains (k_gram_b2; 1: where they fill rounds)
    bool centre_stale = true;
    int tanh_cr = 1;                  // plan option: each net's last hidden layer with the correctly rounded tanh_cr
    int debug_dz = 0;                 // plan option (diagnostics): keep each evaluation's dZ_b / dZ_t
    float* dzb_snap = nullptr;
    float* dzt_snap = nullptr;
    unsigned char* cimgB = nullptr;   // B0 pre-split image (qsplitA_cs bytes)
    unsigned char* cimgT = nullptr;   // T0 pre-split image (qsplitB_cs bytes)
    float* cB0 = nullptr;             // B0 fp32 rows [N][ldz]
    double* ccol = nullptr;           // [112] sum_n B0[n][v]
    double* cysq = nullptr;           // [sum y~^2, sum y~] (the fit guard's scale when centred; d ll / d b0)
    float* cpk = nullptr;             // the centre's packed weights (dp floats)
    unsigned char* cwimg = nullptr;   // ... its forward weight images (wimg_cs bytes, when kept by the scatter)
    unsigned char* cwtimg = nullptr;  // ... its backward W^T images (wtimg_cs bytes)
    float* save_pk = nullptr;         // chain 0's state while the centre is evaluated on its slot
    unsigned char* save_wimg = nullptr;
    unsigned char* save_wtimg = nullptr;
    float* ght_part = nullptr;        // [C][St][49][256] Ht slabs
    float* ghb_part = nullptr;        // [C][Sb][49][256] Hb slabs
    int64_t ght_cs = 0, ghb_cs = 0;
    float* ght = nullptr;             // [C][112][112] Ht
    unsigned char* ghb = nullptr;     // [C][4 blocks] -Hb pre-split
    unsigned char* ghb3 = nullptr;    // [C][4][GRAM_P3_BLOCK] its 4th plane
    bool last_gram = false;       // the last gradient evaluation ran the Gram form (get_option gram: bit 1)
    int last_gram_chains = 0;     // ... for this many of its chains (get_option gram_chains)
    int64_t n_grad_calls = 0;     // DeepONet gradient evaluations (calls) since creation / reset (get_option grad_evals)
    int64_t n_gram_calls = 0;     // ... of which ran the Gram form for some chain (get_option gram_evals)
    int64_t n_gram_chain_evals = 0;   // chain-evaluations in Gram form (get_option gram_chain_evals)
    // Fit guard (plan option gram_guard = k: threshold 10^-k on sum r^2 / sum y^2; 0 = off). The Gram form's two
    // O(|y|) terms cancel to O(|S - y|), so its rounding grows like |y| / |S - y| (profiles/r04_gram_fit_table.json).
    // Every all-residual evaluation (end points, log-prob / value / forward calls) writes each chain's fit ratio and
    // copies it to a pinned 2-slot ring (event per slot); a gradient-only evaluation sends chain c to the residual
    // form when the ratio of its PREVIOUS-BUT-ONE snapshot is below the threshold -- a deterministic function of the
    // chain's own history (two evaluations of lag keep the host one trajectory ahead of the GPU without a stall).
    // Default k = 1 (round 5, profiles/r05_gram_fit_table.json): against fp64, the Gram form's gradient error is 7.7e-4
    // of its norm at fit 0.13 and grows like |y| / |S - y| (8e-3 at 1.5e-3, 6e-2 at 1.5e-5), while the reference's own
    // fp32 closure stays at 5.6e-5 .. 5e-3 and the residual form at 2.3e-4 .. 6e-3 -- so the Gram form runs only where
    // its error stays near 1e-3 (fit >= 0.1) and well-fitting chains keep the residual form.
    int gram_guard = 1;
    // per-item target subsets (VI training with p < P): NaN targets mark the excluded (item, point) pairs, whose
    // residual side A counts as 0; lik_count = the pairs that remain (0: N P). The Gram form and the fit guard are
    // off for a masked plan (their data images and sum y^2 would take the NaNs).
    int y_masked = 0;
    int64_t lik_count = 0;
    float* fit_dev = nullptr;     // [maxC] fit ratios of the last all-residual evaluation
    double* ysq_dev = nullptr;    // [sum y^2, sum y] (k_ysq, whenever the data images are rebuilt)
    double* gcol = nullptr;       // [C][2][112] fp64 column sums of Zb^ / Zt^ (k_gram_sum), the exact d ll / d b0
    double* ysq_part = nullptr;
    float* fit_host = nullptr;    // pinned [2][maxC]
    hipEvent_t fit_ev[2] = {nullptr, nullptr};
    int snap_C[2] = {0, 0};
    int64_t n_snap = 0;
    bool capturing = false;       // inside a hipGraph capture: no snapshot (the ring is host state)
    bool timg_live = false;       // the W^T images hold this evaluation's theta (scatter-kept or split this evaluation)
    bool last_bwd_chain = false;  // the last gradient evaluation ran k_bwd_chain (get_option bwd_chain: bit 1)
    float *g_theta = nullptr, *g_logp = nullptr, *g_grad = nullptr;
    int graph_on = -1;          // -1: follow VIHMC_GRAPH
    // hidden-layer forward products as exact 3-way bf16 splits (6 bf16 MFMA products, fp32 accumulate;
    // fp32-level accuracy, vihmc_fused.hip); VIHMC_FWD_BF16=0 or vihmc_plan_option turns it off
    int fwd_bf16x6 = [] {
        const char* e = std::getenv("VIHMC_FWD_BF16");
        return e ? (std::atoi(e) != 0 ? 1 : 0) : 1;
    }();
    // layer backward in the same form (k_bwd_bf, layers with n_out = 100, n_in <= 112); VIHMC_BWD_BF16=0
    // turns it off. Read at plan creation: it also sizes the backward row chunks (1 workgroup per CU)
    int bwd_bf16x6 = [] {
        const char* e = std::getenv("VIHMC_BWD_BF16");
        return e ? (std::atoi(e) != 0 ? 1 : 0) : 1;
    }();
    // side-A contraction in the same bf16x6 form (k_contract_bf); VIHMC_CONTRACT_BF16=0 turns it off
    int contract_bf16x6 = [] {
        const char* e = std::getenv("VIHMC_CONTRACT_BF16");
        return e ? (std::atoi(e) != 0 ? 1 : 0) : 1;
    }();

    template <typename T>
    int alloc(T** p, int64_t n) {
        void* v = nullptr;
        const size_t sz = std::max<int64_t>(n, 1) * sizeof(T);
        hipError_t e = guard_pages ? vmm_alloc(&v, sz + (canary ? CANARY_BYTES : 0))
                                   : hipMalloc(&v, sz + (canary ? CANARY_BYTES : 0));
        if (e != hipSuccess) return fail(std::string("hipMalloc(") + std::to_string(sz) + "): " + hipGetErrorString(e), (int)e);
        e = hipMemset(v, 0, sz);
        if (e != hipSuccess) return fail(std::string("hipMemset: ") + hipGetErrorString(e), (int)e);
        if (canary) {
            e = hipMemset(static_cast<unsigned char*>(v) + sz, 0xA5, CANARY_BYTES);
            if (e != hipSuccess) return fail(std::string("hipMemset: ") + hipGetErrorString(e), (int)e);
            canaries.push_back(static_cast<unsigned char*>(v) + sz);
        }
        if (!guard_pages) allocs.push_back(v);
        bytes += sz;
        *p = static_cast<T*>(v);
        return 0;
    }
    template <typename T>
    int upload(T** p, const T* host, int64_t n) {
        if (int rc = alloc(p, n)) return rc;
        HIPCHK(hipMemcpy(*p, host, n * sizeof(T), hipMemcpyHostToDevice));
        return 0;
    }
    ~vihmc_plan() {
        for (hipEvent_t e : fit_ev)
            if (e) (void)hipEventDestroy(e);
        if (fit_host) (void)hipHostFree(fit_host);
        for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
        if (cap_stream) (void)hipStreamDestroy(cap_stream);
        for (void* p : allocs) (void)hipFree(p);
        if (!vmm.empty()) (void)hipDeviceSynchronize();
        for (auto& b : vmm) {
            (void)hipMemUnmap(b.base, b.mapped);
            (void)hipMemRelease(b.h);
            // the address range stays reserved (debug runs only): a later plan's buffers never reuse a virtual range
            // a previous plan mapped, so a stale translation cannot make one plan's access land in another's memory
        }
        for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    }

    int timing_begin(int which, hipStream_t s, hipEvent_t* stop, int nlaunch = 1) {
        *stop = nullptr;
        if (!((timing_on >> which) & 1)) return 0;
        if (timing_every > 1 && (n_evals - 1) % timing_every != 0) return 0;
        while (ev_pool.size() < ev_used + 2) {
            // timing only (read after a stream sync): no system-scope release per record -- with it every event
            // left a ~6 us gap (cache write-back) before the next launch, inside the bench's timed region
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
            ev_pool.push_back(e);
        }
        HIPCHK(hipEventRecord(ev_pool[ev_used], s));
        *stop = ev_pool[ev_used + 1];
        ev_cls.resize(ev_used / 2 + 1);
        ev_nl.resize(ev_used / 2 + 1);
        ev_cls[ev_used / 2] = which;
        ev_nl[ev_used / 2] = nlaunch;
        ev_used += 2;
        return 0;
    }
};

namespace vihmc {
int diag_switches() { return VIHMC_DIAG; }   // vihmc_diag.h: one value for every translation unit
}  // namespace vihmc

namespace {

int prior_setup(vihmc_plan* p, const float* prior_mu, const float* prior_sd) {
    std::vector<float> iv(p->K);
    double cst = 0.0;
    const double half_log_2pi = 0.5 * std::log(2.0 * M_PI);
    for (int k = 0; k < p->K; ++k) {
        const double sd = prior_sd[k];
        if (!(sd > 0.0)) return fail("prior_sd must be > 0 (index " + std::to_string(k) + ")");
        iv[k] = (float)(1.0 / (sd * sd));
        cst += -std::log(sd) - half_log_2pi;
    }
    p->prior_const = cst;
    if (int rc = p->upload(&p->prior_mu, prior_mu, p->K)) return rc;
    if (int rc = p->upload(&p->prior_iv, iv.data(), p->K)) return rc;
    return 0;
}

int check_lik(const vihmc_lik_desc& l) {
    if (vihmc::diag_switches()) {
        const char* e = std::getenv("VIHMC_ALLOW_DIAG");
        if (!(e && e[0] == '1'))
            return fail(std::string("library built with timing-only diagnostic switches (") + vihmc_version() +
                        "): results are wrong by design; set VIHMC_ALLOW_DIAG=1 for A/B timing only");
    }
    if (l.loss != VIHMC_LOSS_NLL && l.loss != VIHMC_LOSS_REGRESSION) return fail("unsupported loss kind");
    if (!(l.prior_scale > 0.f)) return fail("prior_scale must be > 0");
    return 0;
}

bool fused_forward_ok(const vihmc_plan* p);
void fused_args(vihmc_plan* p, int C, FusedArgs& a);

// Weight images kept current by the scatter (ScatterImg): per sampled index the byte offsets of its plane element
// and of its fp32 copy (k tail / bias) inside a chain's images; then every chain's images are split once from the
// initial packed weights. Only when the fused forward owns layers 1.. of both nets (otherwise k_split_wimg per
// evaluation, or no images).
int image_maps(vihmc_plan* p, const vihmc_deeponet_desc* d, const int64_t* idx) {
    if (!fused_forward_ok(p)) return 0;
    std::vector<int32_t> fw(p->D, -1), ff(p->D, -1), tw(p->D, -1), tf(p->D, -1);
    int img = 0;
    const vihmc_linear* tabs[2] = {d->branch, d->trunk};
    const int nl[2] = {d->n_branch_layers, d->n_trunk_layers};
    for (int net = 0; net < 2; ++net)
        for (int j = 1; j < nl[net]; ++j, ++img) {
            const vihmc_linear& l = tabs[net][j];
            const int64_t base = (int64_t)img * FWD_WIMG, tbase = (int64_t)img * BWD_WTIMG;
            for (int r = 0; r < l.n_out; ++r) {
                for (int c = 0; c < l.n_in; ++c) {
                    const int64_t f = l.w_off + (int64_t)r * l.n_in + c;
                    fw[f] = (int32_t)(base + fwd_img_plane_off(r, c));
                    if (c >= 96) ff[f] = (int32_t)(base + fwd_img_tail_off(r, c));
                    // W^T image: row i = c, column n = r; n tail W[96 + q][i] at [i][q]
                    tw[f] = (int32_t)(tbase + c * BWD_WTPITCH + 2 * r);
                    if (r >= 96) tf[f] = (int32_t)(tbase + BWD_WTTAIL + 4 * (c * 4 + (r - 96)));
                }
                ff[l.b_off + r] = (int32_t)(base + fwd_img_bias_off(r));
            }
        }
    std::vector<int32_t> sw(p->K), sf(p->K), stw(p->K), stf(p->K);
    for (int k = 0; k < p->K; ++k) {
        sw[k] = fw[idx[k]];
        sf[k] = ff[idx[k]];
        stw[k] = tw[idx[k]];
        stf[k] = tf[idx[k]];
    }
    if (int rc = p->upload(&p->smap_img, sw.data(), p->K)) return rc;
    if (int rc = p->upload(&p->smap_imgf, sf.data(), p->K)) return rc;
    if (p->wtimg) {                                     // (null: no k_bwd_chain for this plan, no W^T images)
        if (int rc = p->upload(&p->smap_timg, stw.data(), p->K)) return rc;
        if (int rc = p->upload(&p->smap_timgf, stf.data(), p->K)) return rc;
    }
    FusedArgs a{};
    fused_args(p, p->maxC, a);
    HIPCHK(launch_split_wimg(a, nullptr));
    if (p->wtimg) HIPCHK(launch_split_wtimg(a, p->wtimg, p->wtimg_cs, nullptr));
    HIPCHK(hipDeviceSynchronize());
    p->img_by_scatter = true;
    return 0;
}

ScatterImg scatter_img(const vihmc_plan* p) {
    return ScatterImg{p->wimg, p->wimg_cs, p->smap_img, p->smap_imgf, fwd_img_plane_stride(),
                      p->wtimg, p->wtimg_cs, p->smap_timg, p->smap_timgf, BWD_WTPLANE};
}

// Gram-form buffers (W = 100 plans): the pre-split data images (built from p->y by gram_images, again whenever the
// data changes) and the per-chain work buffers of vihmc_gram.hip. Split-K of the y Zt^ product: S slabs of SL trunk
// blocks (8 at 16 chains: 512 T_b workgroups of 40 blocks).
int gram_setup(vihmc_plan* p, int C) {
    const int nblkN = cdiv(p->N, CONTRACT_SPLIT_ROWS), nblkP = cdiv(p->P, CONTRACT_SPLIT_ROWS);
    p->gNG = cdiv(p->N, 256);
    p->gPT = cdiv(p->P, 256);
    // split-K of the two data products sized for the plan's chain count, so one launch of each kernel fills the 256
    // CUs: k_gram_a's NG S C T_b + S C Gram-t + C Gram-b units, k_gram_b's PT SB C T_t + C ceil(N/32) dZb units
    // within one round where the chain count allows. At 16 chains: S = 8 (slabs 4 / 8 / 12: 0.499 / 0.496 / 0.523 ms
    // per Gram-form evaluation, profiles/r03z_ab_gram_slabs.txt), SB = 1; at one chain S = 46, SB = 5.
    p->gS = std::max(8, (256 - C) / ((p->gNG + 1) * C));
    p->gS = std::min(p->gS, nblkP);
    p->gSL = cdiv(nblkP, p->gS);
    p->gS = cdiv(nblkP, p->gSL);
    // Gram-t slabs: the T_b split (k_gram_sum adds them up); Gram-b slabs: the branch blocks cut to the same slab
    // length, so no k_gram_a unit runs longer than a T_b unit (one unit of all nblkN blocks at one chain set
    // k_gram_a's time: 45 us, profiles/r04n_c1)
    p->gSt = p->gS;
    p->gSLt = p->gSL;
    // centred: the Gram-t units (H beside G, ~0.8 of a T_b unit) are k_gram_a's short units that fill the chip around the
    // 512 T_b units at 16 chains; shorter ones (GRAM_T_SPLIT slabs per T_b slab) pack the rounds tighter
    p->gSLtc = cdiv(nblkP, std::min(nblkP, p->gS * (C >= 8 ? GRAM_T_SPLIT : 1)));
    p->gStc = cdiv(nblkP, p->gSLtc);
    p->gSLb = std::min(p->gSLtc, nblkN);              // the Gram-t cut (16 chains: slabs of 20 and 12 blocks)
    p->gSb = cdiv(nblkN, p->gSLb);
    const int ngrp = cdiv(p->N, 32);
    p->gSB = std::max(1, std::min(nblkN, (256 - std::min(ngrp * C, 128)) / (p->gPT * C)));
    p->gSLB = cdiv(nblkN, p->gSB);
    p->gSB = cdiv(nblkN, p->gSLB);
    p->gya_ld = 32 * nblkP;
    p->gyb_ld = 32 * nblkN;
    p->gya_plane = (int64_t)p->gNG * 256 * p->gya_ld;
    p->gyb_plane = (int64_t)p->gPT * 256 * p->gyb_ld;
    if (int rc = p->alloc(&p->gya, 3 * p->gya_plane)) return rc;
    if (int rc = p->alloc(&p->gyb, 3 * p->gyb_plane)) return rc;
    p->gtb_cs = (int64_t)p->gS * p->gNG * 8 * 14 * 256;
    if (int rc = p->alloc(&p->gtb_part, p->gtb_cs * C)) return rc;
    p->ggt_part_cs = (int64_t)std::max(p->gSt, p->gStc) * 28 * 256;   // the 28 upper tiles per slab
    if (int rc = p->alloc(&p->ggt_part, p->ggt_part_cs * C)) return rc;
    p->ggb_part_cs = (int64_t)p->gSb * 28 * 256;
    if (int rc = p->alloc(&p->ggb_part, p->ggb_part_cs * C)) return rc;
    // more than GRAM_TB_DIRECT T_b slabs: k_gram_sum adds them up once (fixed order) for the dZb epilogue units
    if (p->gS > GRAM_TB_DIRECT) {
        p->gtbs_cs = (int64_t)p->gNG * 8 * 14 * 256;
        if (int rc = p->alloc(&p->gtb_sum, p->gtbs_cs * C)) return rc;
    }
    if (int rc = p->alloc(&p->ggt, (int64_t)112 * 112 * C)) return rc;
    if (int rc = p->alloc(&p->ggt64, (int64_t)112 * 112 * C)) return rc;
    if (int rc = p->alloc(&p->ggb, (int64_t)4 * CONTRACT_SPLIT_BLOCK * C)) return rc;
    if (int rc = p->alloc(&p->ggb3, (int64_t)4 * GRAM_P3_BLOCK * C)) return rc;
    p->gstats_cs = 2 * (int64_t)p->gPT * 8;
    if (int rc = p->alloc(&p->gstats, p->gstats_cs * C)) return rc;
    if (p->gSB > 1) {
        p->gtt_cs = (int64_t)p->gPT * p->gSB * 8 * 14 * 256;
        if (int rc = p->alloc(&p->gtt_part, p->gtt_cs * C)) return rc;
    }
    if (int rc = p->alloc(&p->fit_dev, C)) return rc;
    if (int rc = p->alloc(&p->ysq_dev, 2)) return rc;           // sum y^2, sum y
    if (int rc = p->alloc(&p->ysq_part, 2 * YSQ_PARTS)) return rc;
    if (int rc = p->alloc(&p->gcol, 4 * 112 * (int64_t)C)) return rc;
    // centred form: the centre's images / rows and column sums, the H slabs and sums, chain 0's save area
    if (int rc = p->alloc(&p->cimgB, p->qsplitA_cs)) return rc;
    if (int rc = p->alloc(&p->cimgT, p->qsplitB_cs)) return rc;
    if (int rc = p->alloc(&p->cB0, (int64_t)p->N * p->ldz)) return rc;
    if (int rc = p->alloc(&p->ccol, 112)) return rc;
    if (int rc = p->alloc(&p->cysq, 2)) return rc;
    p->ght_cs = (int64_t)p->gStc * 49 * 256;
    p->ghb_cs = (int64_t)p->gSb * 49 * 256;
    if (int rc = p->alloc(&p->ght_part, p->ght_cs * C)) return rc;
    if (int rc = p->alloc(&p->ghb_part, p->ghb_cs * C)) return rc;
    if (int rc = p->alloc(&p->ght, (int64_t)112 * 112 * C)) return rc;
    if (int rc = p->alloc(&p->ghb, (int64_t)4 * CONTRACT_SPLIT_BLOCK * C)) return rc;
    if (int rc = p->alloc(&p->ghb3, (int64_t)4 * GRAM_P3_BLOCK * C)) return rc;
    HIPCHK(hipHostMalloc((void**)&p->fit_host, sizeof(float) * 2 * (size_t)C));
    for (auto& e : p->fit_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p->gram_alloc = true;
    return 0;
}

// data images + the fit guard's sum y^2, whenever the plan's data change (the guard's history starts over). Centred
// (gram_center): the images hold y~ and are built with the centre by ensure_centre, before the next evaluation that
// can use them.
int gram_images(vihmc_plan* p, hipStream_t s) {
    if (!p->gram_alloc) return 0;
    HIPCHK(launch_ysq(p->y, (int64_t)p->N * p->P, p->ysq_part, p->ysq_dev, s));
    p->n_snap = 0;
    p->centre_stale = true;
    if (!p->gram_center)
        HIPCHK(launch_gram_yimg(p->y, p->N, p->P, p->gya, p->gya_plane, p->gya_ld, p->gyb, p->gyb_plane, p->gyb_ld, s));
    return 0;
}

int deeponet_forward_layers(vihmc_plan* p, int C, hipStream_t s, bool img, bool gram_only);

// The centre of the centred Gram form: the network output at the centre weights (cpk, the frozen vector) evaluated on
// chain 0's slot -- its packed weights and weight images saved and restored around it, so a state the previous
// gather scattered there survives -- then y~ = y - S0 (fp64, k_center_y) into the G^T scratch, the data images of y~,
// sum y~^2 / sum y~. Called at the start of an evaluation (nothing of it has run yet), outside graph capture.
int ensure_centre(vihmc_plan* p, hipStream_t s) {
    if (!p->gram_alloc || !p->gram_center || !p->centre_stale || !p->cpk) return 0;
    const size_t pkb = sizeof(float) * (size_t)p->dp;
    const bool wi = p->img_by_scatter && p->wimg && p->cwimg;
    const bool wt = p->img_by_scatter && p->wtimg && p->cwtimg;
    HIPCHK(hipMemcpyAsync(p->save_pk, p->packed, pkb, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(p->packed, p->cpk, pkb, hipMemcpyDeviceToDevice, s));
    if (wi) {
        HIPCHK(hipMemcpyAsync(p->save_wimg, p->wimg, (size_t)p->wimg_cs, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(p->wimg, p->cwimg, (size_t)p->wimg_cs, hipMemcpyDeviceToDevice, s));
    }
    if (wt) {
        HIPCHK(hipMemcpyAsync(p->save_wtimg, p->wtimg, (size_t)p->wtimg_cs, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(p->wtimg, p->cwtimg, (size_t)p->wtimg_cs, hipMemcpyDeviceToDevice, s));
    }
    p->img_by_fwd = false;
    if (int rc = deeponet_forward_layers(p, 1, s, true, false)) return rc;
    Net& b = p->nets[0];
    Net& t = p->nets[1];
    if (!p->img_by_fwd) {
        HIPCHK(launch_split_blocks(b.act + b.h_off.back(), b.act_cs, p->ldz, p->N, p->qsplitA, p->qsplitA_cs, 1, s));
        HIPCHK(launch_split_blocks(t.act + t.h_off.back(), t.act_cs, p->ldz, p->P, p->qsplitB, p->qsplitB_cs, 1, s));
        GramArgs ga{};
        ga.bimg = p->qsplitA;
        ga.timg = p->qsplitB;
        ga.b0 = p->packed;
        ga.N = p->N;
        ga.P = p->P;
        ga.C = 1;
        HIPCHK(launch_gram_aug(ga, s));
    }
    p->img_by_fwd = false;
    HIPCHK(hipMemcpyAsync(p->cimgB, p->qsplitA, (size_t)p->qsplitA_cs, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(p->cimgT, p->qsplitB, (size_t)p->qsplitB_cs, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(p->cB0, b.act + b.h_off.back(), sizeof(float) * (size_t)p->N * p->ldz,
                          hipMemcpyDeviceToDevice, s));
    float* yc = p->gT;                                    // scratch: G^T of chain 0 (>= N P floats)
    HIPCHK(launch_center_y(p->y, p->cB0, t.act + t.h_off.back(), p->cpk, p->N, p->P, p->W, p->ldz, yc, p->ccol, s));
    HIPCHK(launch_gram_yimg(yc, p->N, p->P, p->gya, p->gya_plane, p->gya_ld, p->gyb, p->gyb_plane, p->gyb_ld, s));
    HIPCHK(launch_ysq(yc, (int64_t)p->N * p->P, p->ysq_part, p->cysq, s));
    HIPCHK(hipMemcpyAsync(p->packed, p->save_pk, pkb, hipMemcpyDeviceToDevice, s));
    if (wi) HIPCHK(hipMemcpyAsync(p->wimg, p->save_wimg, (size_t)p->wimg_cs, hipMemcpyDeviceToDevice, s));
    if (wt) HIPCHK(hipMemcpyAsync(p->wtimg, p->save_wtimg, (size_t)p->wtimg_cs, hipMemcpyDeviceToDevice, s));
    p->centre_stale = false;
    p->n_snap = 0;                                        // the fit scale changed: the guard's history starts over
    return 0;
}

// the number of (row, point) pairs in the likelihood
double lik_count(const vihmc_plan* p) { return p->lik_count > 0 ? (double)p->lik_count : (double)p->N * (double)p->P; }

bool guard_live(const vihmc_plan* p) {
    return p->gram_alloc && p->gram_guard > 0 && p->maxC <= GUARD_MAXC && !p->capturing && !p->y_masked;
}

// chains of this gradient-only evaluation that run the residual form: previous-but-one snapshot below the threshold
int guard_select(vihmc_plan* p, int C, ChainBits& bits, int& n) {
    n = 0;
    bits = ChainBits{};
    if (!guard_live(p) || p->n_snap < 2) return 0;
    const int k = (int)((p->n_snap - 2) & 1);
    if (p->snap_C[k] != C) return 0;                     // a snapshot of another chain count says nothing here
    HIPCHK(hipEventSynchronize(p->fit_ev[k]));           // normally complete already (one trajectory back)
    const float thr = std::pow(10.f, -(float)p->gram_guard);
    const float* f = p->fit_host + (size_t)k * p->maxC;
    for (int c = 0; c < C; ++c)
        if (f[c] < thr) {
            bits.w[c >> 5] |= 1u << (c & 31);
            ++n;
        }
    return 0;
}

// after an all-residual evaluation wrote fit_dev: copy it into the next ring slot
int guard_snapshot(vihmc_plan* p, int C, hipStream_t s) {
    const int k = (int)(p->n_snap & 1);
    HIPCHK(hipMemcpyAsync(p->fit_host + (size_t)k * p->maxC, p->fit_dev, sizeof(float) * (size_t)C,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(p->fit_ev[k], s));
    p->snap_C[k] = C;
    ++p->n_snap;
    return 0;
}

// The form is a property of the plan (its max_chains), not of the call's chain count: a chain's trajectory does not
// depend on how many chains share its launch (a ragged last rank, a partial batch) -- ADVICE r3.
bool gram_on(const vihmc_plan* p) {
    // a guard that cannot run (more chains than the fit ring holds) keeps the plan on the residual form: the guard
    // exists to keep well-fitting chains off the cancellation-limited Gram gradient
    return p->gram && p->gram_alloc && p->W == 100 && p->contract_bf16x6 && p->maxC >= p->gram_min_chains &&
           !p->y_masked && (p->gram_guard == 0 || p->maxC <= GUARD_MAXC);
}

GramArgs gram_args(vihmc_plan* p, int C) {
    GramArgs a{};
    a.bimg = p->qsplitA;
    a.bimg_cs = p->qsplitA_cs;
    a.nblkN = cdiv(p->N, CONTRACT_SPLIT_ROWS);
    a.timg = p->qsplitB;
    a.timg_cs = p->qsplitB_cs;
    a.nblkP = cdiv(p->P, CONTRACT_SPLIT_ROWS);
    a.ya = p->gya;
    a.ya_plane = p->gya_plane;
    a.ya_ld = p->gya_ld;
    a.yb = p->gyb;
    a.yb_plane = p->gyb_plane;
    a.yb_ld = p->gyb_ld;
    a.tb_part = p->gtb_part;
    a.tb_cs = p->gtb_cs;
    a.gt_part = p->ggt_part;
    a.gt_cs = p->ggt_part_cs;
    a.gb_part = p->ggb_part;
    a.gb_cs = p->ggb_part_cs;
    a.Sb = p->gSb;
    a.SLb = p->gSLb;
    a.tb_sum = p->gtb_sum;
    a.tbs_cs = p->gtbs_cs;
    a.gt = p->ggt;
    a.gt64 = p->ggt64;
    a.gb3img = p->ggb3;
    a.gt_cs2 = 112 * 112;
    a.gbimg = p->ggb;
    a.gbimg_cs = 4 * CONTRACT_SPLIT_BLOCK;
    const Net& b = p->nets[0];
    const Net& t = p->nets[1];
    a.zb = b.act + b.h_off.back();
    a.zb_cs = b.act_cs;
    a.dzb = b.delta[0];
    a.dzb_cs = b.delta_cs;
    a.dzt = t.delta[0];
    a.dzt_cs = t.delta_cs;
    a.stats = p->gstats;
    a.stats_cs = p->gstats_cs;
    a.gcol = p->gcol;
    a.gcol_cs = 4 * 112;
    a.ysum = p->ysq_dev + 1;
    a.center = p->gram_center ? 1 : 0;
    a.pair2 = p->gram_pair2;
    if (a.center) {
        a.cbimg = p->cimgB;
        a.ctimg = p->cimgT;
        a.cb0 = p->cB0;
        a.ccol = p->ccol;
        a.cysum = p->cysq + 1;
        a.ht_part = p->ght_part;
        a.ht_cs = p->ght_cs;
        a.hb_part = p->ghb_part;
        a.hb_cs = p->ghb_cs;
        a.ht = p->ght;
        a.hbimg = p->ghb;
        a.hb3img = p->ghb3;
    }
    a.b0 = p->packed;
    a.b0_cs = p->dp;
    a.N = p->N;
    a.P = p->P;
    a.ldz = p->ldz;
    a.NG = p->gNG;
    a.S = p->gS;
    a.SL = p->gSL;
    a.PT = p->gPT;
    a.St = p->gram_center ? p->gStc : p->gSt;
    a.SLt = p->gram_center ? p->gSLtc : p->gSLt;
    a.SB = p->gSB;
    a.SLB = p->gSLB;
    a.tt_part = p->gtt_part;
    a.tt_cs = p->gtt_cs;
    a.C = C;
    const float v = std::max(p->lik.tau_out, 1e-6f);
    a.gscale = p->lik.loss == VIHMC_LOSS_NLL ? -1.f / v : -p->lik.tau_out;
    return a;
}

// k_reduce grid extent of a job list in max_len units (grid x = span / 256): the x-blocks its jobs use. A block sums
// 256 floats (grouped and scalar forms) or 1,024 (vector / tiled jobs below REDUCE_GROUP_MIN slabs); a grid sized by
// the longest job's floats left up to three quarters of its blocks exiting at once (16 chains: k_reduce 22.9 -> 21.8
// us per launch, profiles/r05s2_span_ab.txt)
constexpr int CONTRACT_B_MIN_Q = 160;   // side-B trunk rows per workgroup, at least (bf16x6 k_contract_bf_b)

int reduce_span(const ReduceJob* jobs, int n) {
    int span = 0;
    for (int i = 0; i < n; ++i) {
        const ReduceJob& J = jobs[i];
        const bool grouped = J.n_parts >= REDUCE_GROUP_MIN;
        int per = 256;
        if (J.tiled) {
            per = grouped ? 256 : 1024;
        } else {
            // k_reduce's own test for the float4 forms
            const bool vec = ((J.len | J.part_stride | J.in_cs | J.dst_cs) & 3) == 0 &&
                             ((reinterpret_cast<uintptr_t>(J.src) | reinterpret_cast<uintptr_t>(J.dst)) & 15) == 0;
            per = vec && !grouped ? 1024 : 256;
        }
        span = std::max(span, 256 * cdiv(J.len, per));
    }
    return span;
}

int build_deeponet(vihmc_plan* p, const vihmc_deeponet_desc* d, const float* xb, const float* tf, const float* y,
                   const float* frozen, const int64_t* idx, const float* prior_mu, const float* prior_sd) {
    if (d->n_branch_layers < 1 || d->n_trunk_layers < 1) return fail("empty branch or trunk");
    if (d->N < 1 || d->P < 1 || d->K < 1 || d->max_chains < 1) return fail("N, P, K, max_chains must be >= 1");
    if (int rc = check_lik(d->lik)) return rc;
    p->kind = 0;
    p->D = d->n_params;
    p->K = d->K;
    p->maxC = d->max_chains;
    p->lik = d->lik;
    p->N = d->N;
    p->P = d->P;

    // ---- layer tables + packed layout --------------------------------------------------------
    std::vector<int32_t> map_w(p->D, -1), map_wt(p->D, -1);
    if (p->D < 1) return fail("n_params must be >= 1");
    map_w[0] = 0;  // scalar output bias b (model.py:26) -> packed slot 0
    int64_t off = 4;
    const vihmc_linear* tabs[2] = {d->branch, d->trunk};
    const int nl[2] = {d->n_branch_layers, d->n_trunk_layers};
    const int in_w[2] = {d->in_branch, d->in_trunk};
    const int rows[2] = {d->N, d->P};
    for (int net = 0; net < 2; ++net) {
        Net& n = p->nets[net];
        n.rows = rows[net];
        n.ld_in = (int)r4(in_w[net]);
        int prev = in_w[net];
        for (int j = 0; j < nl[net]; ++j) {
            const vihmc_linear& l = tabs[net][j];
            if (l.n_in != prev) return fail("layer fan-in does not match the previous fan-out");
            if (l.n_out < 1 || l.n_out > 128 || l.n_in < 1 || l.n_in > 128)
                return fail("layer widths must be in [1, 128]");
            if (l.act < 0 || l.act > 2 || (j == nl[net] - 1 && l.act != VIHMC_ACT_IDENTITY) ||
                (j < nl[net] - 1 && l.act == VIHMC_ACT_IDENTITY))
                return fail("DeepONet layers: tanh/relu hidden activations, identity last layer");
            if (l.b_off < 0) return fail("DeepONet layers need a bias");
            LayerPk L{};
            L.n_out = l.n_out;
            L.n_in = l.n_in;
            L.ldi = (int)r4(l.n_in);
            L.ldo = (int)r4(l.n_out);
            L.act = l.act;
            L.wp = off;
            off += (int64_t)L.n_out * L.ldi;
            L.bias = off;
            off += r4(L.n_out);
            L.wt = off;
            off += (int64_t)L.n_in * L.ldo;
            for (int r = 0; r < l.n_out; ++r) {
                for (int c = 0; c < l.n_in; ++c) {
                    const int64_t f = l.w_off + (int64_t)r * l.n_in + c;
                    if (f < 0 || f >= p->D || map_w[f] != -1) return fail("weight offsets overlap or exceed n_params");
                    map_w[f] = (int32_t)(L.wp + (int64_t)r * L.ldi + c);
                    map_wt[f] = (int32_t)(L.wt + (int64_t)c * L.ldo + r);
                }
                const int64_t fb = l.b_off + r;
                if (fb < 0 || fb >= p->D || map_w[fb] != -1) return fail("bias offsets overlap or exceed n_params");
                map_w[fb] = (int32_t)(L.bias + r);
            }
            n.L.push_back(L);
            prev = l.n_out;
        }
    }
    for (int64_t i = 0; i < p->D; ++i)
        if (map_w[i] < 0) return fail("layer table does not cover parameter " + std::to_string(i));
    p->fmap_host = map_w;
    if (p->nets[0].L.back().n_out != p->nets[1].L.back().n_out)
        return fail("branch and trunk output widths differ");
    p->W = p->nets[0].L.back().n_out;
    p->ldz = (int)r4(p->W);
    p->dp = r64(off);
    if (p->dp >= (int64_t(1) << 31)) return fail("packed layout too large");

    std::vector<int32_t> sw(p->K), swt(p->K);
    for (int k = 0; k < p->K; ++k) {
        const int64_t i = idx[k];
        if (i < 0 || i >= p->D) return fail("sensitive index out of range");
        sw[k] = map_w[i];
        swt[k] = map_wt[i];
    }
    if (int rc = p->upload(&p->smap_w, sw.data(), p->K)) return rc;
    if (int rc = p->upload(&p->smap_wt, swt.data(), p->K)) return rc;
    if (p->K < p->D) {
        // the weight-gradient reduce sums only quads that hold a sampled parameter (bench: K = 10 % of D)
        std::vector<uint8_t> smp((size_t)p->dp, 0);
        for (int k = 0; k < p->K; ++k) smp[(size_t)sw[k]] = 1;
        if (int rc = p->upload(&p->gsamp, smp.data(), p->dp)) return rc;
    }
    if (int rc = prior_setup(p, prior_mu, prior_sd)) return rc;

    const int C = p->maxC;
    if (int rc = p->alloc(&p->packed, p->dp * C)) return rc;
    if (int rc = p->alloc(&p->gp, p->dp * C)) return rc;
    {
        float* d_frozen = nullptr;
        int32_t *d_mw = nullptr, *d_mwt = nullptr;
        std::vector<void*> tmp;
        HIPCHK(hipMalloc((void**)&d_frozen, p->D * sizeof(float)));
        HIPCHK(hipMalloc((void**)&d_mw, p->D * sizeof(int32_t)));
        HIPCHK(hipMalloc((void**)&d_mwt, p->D * sizeof(int32_t)));
        HIPCHK(hipMemcpy(d_frozen, frozen, p->D * sizeof(float), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_mw, map_w.data(), p->D * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d_mwt, map_wt.data(), p->D * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(launch_init_packed(p->packed, p->dp, C, d_frozen, d_mw, d_mwt, p->D, nullptr));
        HIPCHK(hipDeviceSynchronize());
        (void)hipFree(d_frozen);
        (void)hipFree(d_mw);
        (void)hipFree(d_mwt);
    }

    // ---- shared inputs ---------------------------------------------------------------------------
    const float* inputs[2] = {xb, tf};
    for (int net = 0; net < 2; ++net) {
        Net& n = p->nets[net];
        std::vector<float> pad((size_t)n.rows * n.ld_in, 0.f);
        for (int r = 0; r < n.rows; ++r)
            std::memcpy(&pad[(size_t)r * n.ld_in], inputs[net] + (size_t)r * in_w[net], in_w[net] * sizeof(float));
        if (int rc = p->upload(&n.input, pad.data(), (int64_t)pad.size())) return rc;
    }
    const int64_t NP = (int64_t)p->N * p->P;
    if (int rc = p->upload(&p->y, y, NP)) return rc;
    p->ldgT = (int)((p->N + 31) / 32 * 32);
    p->gT_cs = r64((int64_t)(p->P + 1) * p->ldgT);      // the bf16x6 blocked layout uses (P rounded even) rows
    if (int rc = p->alloc(&p->gT, p->gT_cs * C)) return rc;
    if (p->W == 100) {
        // pre-split weight images of the bf16x6 fused forward (layers 1.. of both nets)
        p->wimg_cs = (int64_t)(p->nets[0].L.size() - 1 + p->nets[1].L.size() - 1) * FWD_WIMG;
        if (int rc = p->alloc(&p->wimg, p->wimg_cs * C)) return rc;
        p->qsplitA_cs = (int64_t)cdiv(p->N, CONTRACT_SPLIT_ROWS) * CONTRACT_SPLIT_BLOCK;
        if (int rc = p->alloc(&p->qsplitA, p->qsplitA_cs * C)) return rc;
        p->qsplitB_cs = (int64_t)cdiv(p->P, CONTRACT_SPLIT_ROWS) * CONTRACT_SPLIT_BLOCK;
        if (int rc = p->alloc(&p->qsplitB, p->qsplitB_cs * C)) return rc;
        if (int rc = gram_setup(p, C)) return rc;
    }

    // ---- per-chain work buffers ---------------------------------------------------------------------
    for (int net = 0; net < 2; ++net) {
        Net& n = p->nets[net];
        int64_t a = 0;
        int maxld = 0;
        for (auto& L : n.L) {
            n.h_off.push_back(a);
            a += (int64_t)n.rows * L.ldo;
            maxld = std::max(maxld, L.ldo);
        }
        n.act_cs = r64(a);
        if (int rc = p->alloc(&n.act, n.act_cs * C)) return rc;
        n.delta_cs = r64((int64_t)n.rows * maxld);
        for (int b = 0; b < 2; ++b)
            if (int rc = p->alloc(&n.delta[b], n.delta_cs * C)) return rc;
        // weight-gradient partial slabs: one per row chunk
        // fused-backward row chunk: one workgroup per chunk, sized so a max_chains launch over both
        // nets is ~one resident round (k_bwd_ws: 2 workgroups/CU x 256 CUs, ~68 KB of LDS; k_bwd_bf:
        // 1 workgroup/CU, 87 KB of LDS and 256-VGPR waves)
        {
            const int64_t rows_all = (int64_t)p->nets[0].rows + p->nets[1].rows;
            // two 512-thread workgroups per CU, 32-row sub-tiles; the chunk R (a multiple of the sub-tile)
            // is the smallest for which both nets' workgroups of all max_chains chains fit one resident round
            const int slots = p->bwd_bf16x6 ? 256 : 512, sub = BWD_SUB;
            const int64_t r_b = p->nets[0].rows, r_t = p->nets[1].rows;
            int64_t R = std::max<int64_t>(sub, (cdiv((int64_t)C * rows_all, slots) + sub - 1) / sub * sub);
            while ((int64_t)C * (cdiv(r_b, R) + cdiv(r_t, R)) > slots && R < rows_all) R += sub;
            // the whole-network backward (k_bwd_chain) runs 64-row chunks: taken whenever they still fit one round
            const int64_t rc = bwd_chain_rows();
            if (p->bwd_bf16x6 && R < rc && (int64_t)C * (cdiv(r_b, rc) + cdiv(r_t, rc)) <= slots) R = rc;
            n.rows_per_chunk = (int)R;
        }
        int64_t po = 0;
        for (size_t j = 0; j < n.L.size(); ++j) {
            LayerPk& L = n.L[j];
            // the input layer has no dX: its launch is dW only, and the branch input layer (K = 101: all seven
            // column tiles) is ~7x the work per row of the trunk one (K = 5: one tile) -- with the common chunk
            // the branch workgroups alone set that launch (41 us of 64-us-class launches at C = 16). Its chunks
            // are cut to VIHMC_BWD_L0_ROWS rows (default 128: 4 sub-tiles) so they fit beside the trunk ones.
            L.rows_per_chunk = n.rows_per_chunk;
            if (j == 0 && L.n_in >= 64) L.rows_per_chunk = std::min(n.rows_per_chunk, 128);
            L.n_chunks = cdiv(n.rows, L.rows_per_chunk);
            // row-major (fp32 backward) or tiled (bf16x6 backward kernels, bwd_tile_off) slabs: room for either
            L.part_stride = r4(std::max<int64_t>((int64_t)L.n_out * L.ldi + L.n_out, bwd_tile_floats((L.ldi + 16) >> 4)));
            L.part_off = po;
            po += L.part_stride * L.n_chunks;
        }
        n.dwpart_cs = r64(po);
        if (int rc = p->alloc(&n.dwpart, n.dwpart_cs * C)) return rc;
    }
    // the whole-network backward's W^T images (k_bwd_chain), only for plans whose backward chunks can be its 64 rows:
    // at larger chain counts nothing reads them, and the scatter would keep them current for nothing (four of its
    // ~ten scattered stores per sampled weight)
    if (p->W == 100) {
        bool chain_rows = true;
        for (int net = 0; net < 2; ++net)
            for (const LayerPk& L : p->nets[net].L) chain_rows &= L.rows_per_chunk == bwd_chain_rows();
        if (chain_rows) {
            p->wtimg_cs = (int64_t)(p->nets[0].L.size() - 1 + p->nets[1].L.size() - 1) * BWD_WTIMG;
            if (int rc = p->alloc(&p->wtimg, p->wtimg_cs * C)) return rc;
        }
    }
    // contraction side B (branch-owner) partials over trunk chunks
    {
        // side A: workgroups own 128 trunk rows and sweep the branch rows; split the sweep (partial
        // dZ_trunk slabs + fixed-order reduce) only when too few workgroups would fill the chip
        const int og_a = cdiv(p->P, CONTRACT_OWN_PER_WG), og_b = cdiv(p->N, CONTRACT_OWN_PER_WG);
        // q-split count: fewest resident rounds x chunks per workgroup (+2 chunks of per-workgroup prologue), one
        // 1024-thread workgroup per CU (single chain: 3 splits of 11 chunks, 240 workgroups in one round)
        int qa = 1;
        {
            const int64_t nch = cdiv(p->N, CONTRACT_SPLIT_ROWS);
            int64_t best = INT64_MAX;
            for (int q = 1; q <= 8; ++q) {
                const int64_t cost = cdiv((int64_t)C * og_a * q, 256) * (cdiv(nch, q) + 2);
                if (cost < best) best = cost, qa = q;
            }
        }
        // multiple of 32 rows: whole blocks of the pre-split image for k_contract_bf (and 16-row chunks)
        p->qperA = (int)(((int64_t)cdiv(p->N, qa) + CONTRACT_SPLIT_ROWS - 1) / CONTRACT_SPLIT_ROWS * CONTRACT_SPLIT_ROWS);
        p->qchunksA = cdiv(p->N, p->qperA);
        if (p->qchunksA > 1) {
            p->partA_cs = r64((int64_t)p->qchunksA * p->P * p->ldz);
            if (int rc = p->alloc(&p->partA, p->partA_cs * C)) return rc;
        }
        // side B: workgroups own 128 branch rows, the trunk sweep is split to match side A's grid
        int qc = std::max(1, (int)std::lround((double)og_a * p->qchunksA / og_b));
        if (p->W == 100) {
            // bf16x6 side B (k_contract_bf_b, 256 owner rows, 1 workgroup per CU): ~256 workgroups
            qc = std::max(1, (int)std::lround(256.0 / ((double)C * cdiv(p->N, CONTRACT_BF_B_OWN))));
            // at least CONTRACT_B_MIN_Q trunk rows per workgroup: below that its time is its prologue, and every further
            // chunk adds an N x ldz partial slab to the reduce (config 4's N = 500 shards: 128 slabs of 80 rows,
            // 28.7 MB for a 0.2-MB result)
            qc = std::min(qc, std::max(1, cdiv(p->P, CONTRACT_B_MIN_Q)));
            qc = std::min(qc, cdiv(p->P, CONTRACT_SPLIT_ROWS));
        }
        p->qperB = (int)(((int64_t)cdiv(p->P, qc) + CONTRACT_SPLIT_ROWS - 1) / CONTRACT_SPLIT_ROWS * CONTRACT_SPLIT_ROWS);
        p->qchunksB = cdiv(p->P, p->qperB);
        p->partB_cs = r64((int64_t)p->qchunksB * p->N * p->ldz);
        if (int rc = p->alloc(&p->partB, p->partB_cs * C)) return rc;
        p->nwavesA = p->qchunksA * og_a * 8;   // stats slots: 8 S waves per workgroup (k_contract_bf;
                                               // the fp32 kernels fill 4 of them)
        p->stats_cs = 2 * (int64_t)p->nwavesA;
        if (int rc = p->alloc(&p->stats, p->stats_cs * C)) return rc;
        if (int rc = p->alloc(&p->lik_buf, C)) return rc;
        if (int rc = p->alloc(&p->lp_part, (int64_t)C * GATHER_SPLIT_MAX)) return rc;
        if (int rc = p->alloc(&p->fin_cnt, C)) return rc;
    }
    // reduce jobs
    {
        ReduceJob jb{};
        jb.src = p->partB;
        jb.in_cs = p->partB_cs;
        jb.part_stride = (int64_t)p->N * p->ldz;
        jb.n_parts = p->qchunksB;
        jb.len = p->N * p->ldz;
        jb.dst = p->nets[0].delta[0];
        jb.dst_cs = p->nets[0].delta_cs;
        p->lenB = jb.len;
        p->spanB = reduce_span(&jb, 1);
        if (int rc = p->upload(&p->jobsB, &jb, 1)) return rc;
        if (p->qchunksA > 1) {
            ReduceJob ja{};
            ja.src = p->partA;
            ja.in_cs = p->partA_cs;
            ja.part_stride = (int64_t)p->P * p->ldz;
            ja.n_parts = p->qchunksA;
            ja.len = p->P * p->ldz;
            ja.dst = p->nets[1].delta[0];
            ja.dst_cs = p->nets[1].delta_cs;
            p->lenA = ja.len;
            // both contraction reduces in one launch (independent outputs: branch and trunk deltas)
            const ReduceJob both[2] = {jb, ja};
            p->spanA = reduce_span(both, 2);
            if (int rc = p->upload(&p->jobsA, both, 2)) return rc;
        }
        // two job lists over the same slabs: row-major (fp32 backward) and, for the layers the bf16x6 kernels run
        // (bwd_bf_ok per launch: layer i from the top of both nets), tiled
        std::vector<ReduceJob> jw, jt;
        std::vector<char> tiled[2];
        for (int net = 0; net < 2; ++net) tiled[net].assign(p->nets[net].L.size(), 0);
        const int maxl = (int)std::max(p->nets[0].L.size(), p->nets[1].L.size());
        for (int i = 0; i < maxl; ++i) {
            BwdArgs ba{};
            int js[2] = {-1, -1};
            for (int net = 0; net < 2; ++net) {
                const Net& n = p->nets[net];
                const int j = (int)n.L.size() - 1 - i;
                if (j < 0) continue;
                js[net] = j;
                const LayerPk& L = n.L[j];
                BwdProb& q = ba.p[ba.nprob++];
                q.ldd = q.ldw = L.ldo;
                q.ldh = L.ldi;
                q.n_out = L.n_out;
                q.n_in = L.n_in;
                q.has_dx = j >= 1;
                q.rows_per_wg = L.rows_per_chunk;
            }
            if (bwd_bf_ok(ba))
                for (int net = 0; net < 2; ++net)
                    if (js[net] >= 0) tiled[net][js[net]] = 1;
        }
        for (int net = 0; net < 2; ++net) {
            Net& n = p->nets[net];
            for (size_t li = 0; li < n.L.size(); ++li) {
                const LayerPk& L = n.L[li];
                ReduceJob j{};
                j.src = n.dwpart + L.part_off;
                j.in_cs = n.dwpart_cs;
                j.part_stride = L.part_stride;
                j.n_parts = L.n_chunks;
                j.len = L.n_out * L.ldi + L.n_out;
                j.dst = p->gp + L.wp;
                j.dst_cs = p->dp;
                // only jobs over many slabs (one or two chains: ~160 row chunks per trunk layer) gain from skipping the
                // unsampled quads; with a few slabs per chain (16 chains) the mask's own loads cost more than the
                // skipped slab loads (k_reduce 22.7 -> 26.9 us per launch, profiles/r05sb_samp_ab.txt)
                j.samp = p->gsamp && L.n_chunks >= REDUCE_GROUP_MIN ? p->gsamp + L.wp : nullptr;
                p->max_lenW = std::max(p->max_lenW, j.len);
                jw.push_back(j);
                if (tiled[net][li]) {
                    j.tiled = 1;
                    j.ntj = (L.ldi + 16) >> 4;
                    j.len = bwd_tile_floats(j.ntj);
                    j.n_out = L.n_out;
                    j.n_in = L.n_in;
                    j.ldi = L.ldi;
                    p->max_lenW = std::max(p->max_lenW, j.len);
                }
                jt.push_back(j);
            }
        }
        p->n_jobsW = (int)jw.size();
        p->spanW = reduce_span(jw.data(), (int)jw.size());
        p->spanWt = reduce_span(jt.data(), (int)jt.size());
        if (int rc = p->upload(&p->jobsW, jw.data(), (int64_t)jw.size())) return rc;
        if (int rc = p->upload(&p->jobsWt, jt.data(), (int64_t)jt.size())) return rc;
    }
    // weight images maintained by the scatter (after the activation layout, which fused_args reads)
    if (p->wimg)
        if (int rc = image_maps(p, d, idx)) return rc;
    if (p->gram_alloc) {
        // the centred Gram form's centre: chain 0's packed weights (and images) now, i.e. the frozen vector
        if (int rc = p->alloc(&p->cpk, p->dp)) return rc;
        if (int rc = p->alloc(&p->save_pk, p->dp)) return rc;
        HIPCHK(hipMemcpy(p->cpk, p->packed, sizeof(float) * (size_t)p->dp, hipMemcpyDeviceToDevice));
        if (p->wimg && p->img_by_scatter) {
            if (int rc = p->alloc(&p->cwimg, p->wimg_cs)) return rc;
            if (int rc = p->alloc(&p->save_wimg, p->wimg_cs)) return rc;
            HIPCHK(hipMemcpy(p->cwimg, p->wimg, (size_t)p->wimg_cs, hipMemcpyDeviceToDevice));
        }
        if (p->wtimg && p->img_by_scatter) {
            if (int rc = p->alloc(&p->cwtimg, p->wtimg_cs)) return rc;
            if (int rc = p->alloc(&p->save_wtimg, p->wtimg_cs)) return rc;
            HIPCHK(hipMemcpy(p->cwtimg, p->wtimg, (size_t)p->wtimg_cs, hipMemcpyDeviceToDevice));
        }
    }
    if (int rc = gram_images(p, nullptr)) return rc;
    HIPCHK(hipDeviceSynchronize());
    return 0;
}

inline int nt_of(int n) { return (n + 15) / 16; }

// row tiles per row-dot workgroup: the whole launch (all problems, all chains) fits one resident round of
// ~3 workgroups per CU (the staged 100x100 weight block is ~42 KB of LDS), so every workgroup stages its
// weights once and no second, partly empty round is left
inline int rowdot_tpw(int64_t total_tiles) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(8, cdiv(total_tiles, (int64_t)768)));
}


// Layers 1..L-1 of both nets can run in the fused register-resident forward (vihmc_fused.hip) when they
// are all 100 -> 100 with the packed [W | bias] block contiguous.
bool fused_forward_ok(const vihmc_plan* p) {
    if (!VIHMC_FUSED_FWD) return false;
    for (int net = 0; net < 2; ++net) {
        const Net& n = p->nets[net];
        const int nl = (int)n.L.size();
        if (nl < 2 || nl - 1 > FUSED_MAXL || n.L[0].ldo < 100) return false;
        for (int j = 1; j < nl; ++j) {
            const LayerPk& L = n.L[j];
            if (L.n_in != 100 || L.n_out != 100 || L.ldi != 100 || L.ldo != 100 || L.bias != L.wp + 100 * 100)
                return false;
        }
    }
    return true;
}

// the forward epilogue's activation code of layer j of a net: each net's last hidden tanh layer runs the correctly
// rounded tanh_cr (plan option tanh_cr, default 1; vihmc_internal.h), every other layer its own activation
int fwd_act(const vihmc_plan* p, const Net& n, int j) {
    const int a = n.L[j].act;
    return a == ACT_TANH && p->tanh_cr && j == (int)n.L.size() - 2 ? (int)ACT_TANH_CR : a;
}

void fused_args(vihmc_plan* p, int C, FusedArgs& a) {
    a.C = C;
    a.packed = p->packed;
    a.dp = p->dp;
    for (int net = 0; net < 2; ++net) {
        Net& n = p->nets[net];
        FusedNet& f = a.net[net];
        f.in = n.act + n.h_off[0];
        f.in_cs = n.act_cs;
        f.ldin = n.L[0].ldo;
        f.out = n.act;
        f.out_cs = n.act_cs;
        f.ldo = 100;
        f.nl = (int)n.L.size() - 1;
        for (int j = 1; j < (int)n.L.size(); ++j) {
            f.h_off[j - 1] = n.h_off[j];
            f.w_off[j - 1] = n.L[j].wp;
            f.act[j - 1] = fwd_act(p, n, j);
        }
        f.rows = n.rows;
    }
    a.net[0].wimg = p->wimg;
    a.net[1].wimg = p->wimg ? p->wimg + (int64_t)a.net[0].nl * FWD_WIMG : nullptr;
    a.net[0].wimg_cs = a.net[1].wimg_cs = p->wimg_cs;
}

// the input layers of both nets can run inside the bf16x6 forward's launch (FusedNet::x): the pre-split-image form
// and an input layer of a shape it stages
bool fused_input_ok(const vihmc_plan* p) {
    if (!p->fwd_bf16x6 || !p->fwd_wimg || !p->wimg || !fwd_fused_bf_needs_wimg() || !p->fwd_in0) return false;
    if ((p->dp & 3) != 0) return false;
    for (int net = 0; net < 2; ++net) {
        const Net& n = p->nets[net];
        const LayerPk& L = n.L[0];
        if (L.n_out != 100 || (L.wp & 3) != 0 || L.ldo < 100 || !fwd_fused_in0_ok(L.n_in, n.ld_in, L.ldi)) return false;
    }
    return true;
}

int launch_forward_fused(vihmc_plan* p, int C, hipStream_t s, bool img, bool in0, bool gram_only) {
    FusedArgs a{};
    fused_args(p, C, a);
    if (in0) {
        for (int net = 0; net < 2; ++net) {
            const Net& n = p->nets[net];
            const LayerPk& L = n.L[0];
            FusedNet& f = a.net[net];
            f.x = n.input;
            f.ldx = n.ld_in;
            f.k0 = L.n_in;
            f.ldw0 = L.ldi;
            f.act0 = fwd_act(p, n, 0);
            f.w0_off = L.wp;
            f.b0_off = L.bias;
        }
    }
    a.net[0].wimg = a.net[1].wimg = nullptr;           // set below when the bf16x6 kernel stages them
    // 12-wave workgroups (one per CU, 84 KB LDS) unless that grid would leave most of the 256 CUs idle
    const int64_t blocks12 = (int64_t)C * (cdiv(p->nets[0].rows, 192) + cdiv(p->nets[1].rows, 192));
    const int nw = blocks12 >= 192 ? 12 : 4;
    // bf16x6 at 12 waves, or at 4 for small chain counts
    const int nwb = nw == 12 ? fwd_fused_bf_waves() : 4;
    if (p->fwd_bf16x6 && (!fwd_fused_bf_needs_wimg() || (p->fwd_wimg && p->wimg))) {
        for (int net = 0; net < 2; ++net) a.net[net].nblk = cdiv(p->nets[net].rows, 16 * nwb);
        if (img) {
            // the contraction's pre-split images of the branch (side A) and trunk (side B) outputs
            a.net[0].qimg = p->qsplitA;
            a.net[0].qimg_cs = p->qsplitA_cs;
            a.net[1].qimg = p->qsplitB;
            a.net[1].qimg_cs = p->qsplitB_cs;
            if (p->gram_alloc) {                           // the Gram form's augmented outputs [Z_b | 1], [Z_t | b0]
                a.net[0].aug = 1;
                a.net[1].aug = 2;
            }
            // an all-Gram evaluation reads the trunk's outputs only through this image (the branch's fp32 rows feed
            // its dZ_b epilogue): their fp32 copy is not stored
            a.net[1].skip_last = gram_only && p->skip_zt ? 1 : 0;
            p->img_by_fwd = true;
        }
        if (p->fwd_wimg && p->wimg) {
            // pre-split weight images, DMA-staged by the forward (FWD_WIMG bytes per fused layer); kept current by the
            // scatter when the plan built its image maps, else split here from the packed weights
            a.net[0].wimg = p->wimg;
            a.net[1].wimg = p->wimg + (int64_t)a.net[0].nl * FWD_WIMG;
            a.net[0].wimg_cs = a.net[1].wimg_cs = p->wimg_cs;
            if (!p->img_by_scatter) {
                HIPCHK(launch_split_wimg(a, s));
                if (p->wtimg) {
                    HIPCHK(launch_split_wtimg(a, p->wtimg, p->wtimg_cs, s));
                    p->timg_live = true;
                }
            }
        }
        HIPCHK(launch_fwd_fused_bf(a, nwb, s));
        return 0;
    }
    for (int net = 0; net < 2; ++net) a.net[net].nblk = cdiv(p->nets[net].rows, 16 * nw);
    HIPCHK(launch_fwd_fused(a, nw, s));
    return 0;
}

// Forward through both MLPs (grouped launches: branch + trunk layer j together); the hidden 100 -> 100
// stack goes through the fused kernel when its shape allows.
int deeponet_forward_layers(vihmc_plan* p, int C, hipStream_t s, bool img, bool gram_only) {
    const int maxl = (int)std::max(p->nets[0].L.size(), p->nets[1].L.size());
    const bool fused = fused_forward_ok(p);
    const bool in0 = fused && fused_input_ok(p);     // the input layers inside the forward's launch
    for (int j = 0; j < maxl; ++j) {
        if ((j == 1 && fused) || in0) {
            hipEvent_t stop = nullptr;
            if (int rc = p->timing_begin(VIHMC_T_FWD, s, &stop)) return rc;
            if (int rc = launch_forward_fused(p, C, s, img, in0, gram_only)) return rc;
            if (stop) HIPCHK(hipEventRecord(stop, s));
            return 0;
        }
        RowdotArgs a{};
        a.C = C;
        int nt = 1;
        int64_t wgs = 0;
        for (int net = 0; net < 2; ++net) {
            Net& n = p->nets[net];
            if (j < (int)n.L.size()) wgs += (int64_t)C * cdiv(n.rows, ROWDOT_WAVES * 32);
        }
        const int ms = wgs >= 512 ? 2 : 1;
        int64_t total_tiles = 0;
        for (int net = 0; net < 2; ++net)
            if (j < (int)p->nets[net].L.size()) total_tiles += (int64_t)C * cdiv(p->nets[net].rows, ROWDOT_WAVES * 16 * ms);
        const int tpw = rowdot_tpw(total_tiles);
        for (int net = 0; net < 2; ++net) {
            Net& n = p->nets[net];
            if (j >= (int)n.L.size()) continue;
            const LayerPk& L = n.L[j];
            RowdotProb& q = a.p[a.nprob++];
            q.A = j == 0 ? n.input : n.act + n.h_off[j - 1];
            q.a_cs = j == 0 ? 0 : n.act_cs;
            q.lda = j == 0 ? n.ld_in : n.L[j - 1].ldo;
            q.B = p->packed + L.wp;
            q.b_cs = p->dp;
            q.ldb = L.ldi;
            q.O = n.act + n.h_off[j];
            q.o_cs = n.act_cs;
            q.ldo = L.ldo;
            q.bias = p->packed + L.bias;
            q.bias_cs = p->dp;
            q.M = n.rows;
            q.Nn = L.n_out;
            q.K = L.n_in;
            q.act = fwd_act(p, n, j);
            q.ntiles = cdiv(n.rows, ROWDOT_WAVES * 16 * ms);
            // long contractions (the branch input layer: K = 101 on the f32 MFMA) one tile per workgroup: with
            // two they set the launch, 45 -> 35.5 us (the trunk input layer, K = 5, shares it at two tiles per
            // workgroup; the two nets as separate launches took 17 + 30 us)
            q.tpw = L.n_in >= 64 && j == 0 ? 1 : tpw;
            q.tiles = cdiv(q.ntiles, q.tpw);
            nt = std::max(nt, nt_of(L.n_out));
        }
        if (a.nprob == 1) a.p[1] = a.p[0];
        HIPCHK(launch_rowdot(a, nt, ms, MODE_FWD, s));
    }
    return 0;
}

// rows per 16-row block of the bf16x6 G^T hand-off, even: every block (16 x 64 B per row) starts on a 128-B line,
// so side A's 1-KB tile stores are whole lines (an odd count left every other block's tiles straddling two
// partial lines, which the memory side read back: +200 MB of fetch per side-A launch at 16 chains)
inline int gt_block_rows(const vihmc_plan* p) { return (p->P + 1) & ~1; }

ContractProb side_a(vihmc_plan* p, int C, bool grad, float* out) {
    Net& b = p->nets[0];
    Net& t = p->nets[1];
    ContractProb q{};
    q.Own = t.act + t.h_off.back();
    q.own_cs = t.act_cs;
    q.ldown = p->ldz;
    q.Q = b.act + b.h_off.back();
    q.q_cs = b.act_cs;
    q.ldq = p->ldz;
    q.Y = p->y;
    q.ldy = p->P;
    q.masked = p->y_masked;
    q.b0 = p->packed;
    q.b0_cs = p->dp;
    if (grad) {
        q.out = p->qchunksA > 1 ? p->partA : t.delta[0];
        q.out_cs = p->qchunksA > 1 ? p->partA_cs : t.delta_cs;
        q.ldout = p->ldz;
        q.out_chunk_stride = p->qchunksA > 1 ? (int64_t)p->P * p->ldz : 0;
        q.gout = p->gT;
        q.gout_cs = p->gT_cs;
        q.ldg = p->contract_bf16x6 && p->W == 100 ? gt_block_rows(p) : p->ldgT;   // bf16x6: 16-row blocked
    } else {
        q.out = out ? out : p->lik_buf;   // dummy when not writing S
        q.out_cs = out ? (int64_t)p->N * p->P : 0;
        q.ldout = p->P;
        q.write_s = out ? 1 : 0;
    }
    q.stats = p->stats;
    q.stats_cs = p->stats_cs;
    q.Mo = p->P;
    q.Mq = p->N;
    q.W = p->W;
    q.o_tiles = cdiv(p->P, CONTRACT_OWN_PER_WG);
    q.q_chunks = p->qchunksA;
    q.q_per_chunk = p->qperA;
    q.with_stats = 1;
    q.bf16x6 = grad && p->W == 100 ? p->contract_bf16x6 : 0;
    q.qimg = p->qsplitA;
    q.qimg_cs = p->qsplitA_cs;
    const float v = std::max(p->lik.tau_out, 1e-6f);
    q.gscale = p->lik.loss == VIHMC_LOSS_NLL ? -1.f / v : -p->lik.tau_out;
    (void)C;
    return q;
}

int deeponet_eval_body(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, float* out,
                       hipStream_t s, const LeapArgs* leap);

int deeponet_eval(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, float* out, hipStream_t s,
                  const LeapArgs* leap = nullptr) {
    if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
    ++p->n_evals;
    hipEvent_t stop = nullptr;
    if (int rc = p->timing_begin(VIHMC_T_EVAL, s, &stop)) return rc;
    if (int rc = deeponet_eval_body(p, theta, C, logp, grad, out, s, leap)) return rc;
    if (stop) HIPCHK(hipEventRecord(stop, s));
    return 0;
}

// k_bwd_chain's arguments when this plan's backward chunks are its 64 rows in every layer of both nets
bool bwd_chain_args(vihmc_plan* p, int C, BwdChainArgs& a) {
    a.C = C;
    for (int net = 0; net < 2; ++net) {
        Net& n = p->nets[net];
        BwdChainNet& cn = a.net[net];
        cn.nl = (int)n.L.size();
        if (cn.nl > BWD_CHAIN_MAXL) return false;
        cn.M = n.rows;
        cn.n_wg = cdiv(n.rows, bwd_chain_rows());
        cn.tanh_all = 1;
        for (int j = 0; j + 1 < cn.nl; ++j) cn.tanh_all &= n.L[j].act == ACT_TANH ? 1 : 0;
        cn.D = n.delta[0];
        cn.d_cs = n.delta_cs;
        cn.ldd = n.L.back().ldo;
        cn.dwpart = n.dwpart;
        cn.dwpart_cs = n.dwpart_cs;
        cn.wtimg = p->wtimg + (net ? (int64_t)(p->nets[0].L.size() - 1) * BWD_WTIMG : 0);
        cn.wtimg_cs = p->wtimg_cs;
        for (int j = 0; j < cn.nl; ++j) {
            const LayerPk& L = n.L[j];
            if (L.rows_per_chunk != bwd_chain_rows() || L.n_chunks != cn.n_wg) return false;
            BwdChainLayer& q = cn.L[j];
            q.H = j == 0 ? n.input : n.act + n.h_off[j - 1];
            q.h_cs = j == 0 ? 0 : n.act_cs;
            q.ldh = L.ldi;
            q.n_in = L.n_in;
            q.n_out = L.n_out;
            q.act = j >= 1 ? n.L[j - 1].act : 0;
            q.part_off = L.part_off;
            q.part_stride = (int32_t)L.part_stride;
        }
    }
    return bwd_chain_ok(a);
}

int deeponet_eval_body(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, float* out,
                       hipStream_t s, const LeapArgs* leap) {
    // the centred Gram form's centre (data images of y~, the fit guard's scale), before anything of this evaluation
    if (gram_on(p) && !p->capturing)
        if (int rc = ensure_centre(p, s)) return rc;
    const ScatterImg si = scatter_img(p);
    if (!(leap && leap->scattered_in))
        HIPCHK(launch_scatter(p->packed, p->dp, C, theta, p->K, p->smap_w, p->smap_wt, s, p->img_by_scatter ? &si : nullptr));
    const bool want_grad = grad != nullptr && out == nullptr;
    // the pre-split contraction images (bf16x6 sides, gradient evaluations) are written by the fused forward
    // when it runs; otherwise k_split_blocks makes them below
    p->img_by_fwd = false;
    p->timg_live = p->img_by_scatter && p->wtimg;      // the scatter above kept the W^T images current
    // gradient-only evaluations (no log-prob returned): the Gram-form contraction, which forms no residual; the fit
    // guard sends the chains whose fit is too good for its cancellation to the residual form (both forms in one
    // evaluation, each launch skipping the other form's chains)
    const bool gram_elig = want_grad && logp == nullptr && gram_on(p);
    ChainBits resid{};
    int n_resid = 0;
    if (gram_elig)
        if (int rc = guard_select(p, C, resid, n_resid)) return rc;
    const bool gram = gram_elig && n_resid < C;          // some chain runs the Gram form
    const bool resid_any = !gram;                        // ... or every chain the residual form
    const bool mixed = gram && n_resid > 0;
    if (int rc = deeponet_forward_layers(p, C, s, want_grad && p->contract_bf16x6 && p->W == 100, gram && !mixed))
        return rc;
    p->last_gram = gram;
    p->last_gram_chains = gram ? C - n_resid : 0;
    if (want_grad) {
        ++p->n_grad_calls;
        if (gram) ++p->n_gram_calls;
        if (gram) p->n_gram_chain_evals += C - n_resid;
    }
    int stats_waves = 0, stats_waves_res = 0;
    if (gram) {
        Net& b = p->nets[0];
        Net& t = p->nets[1];
        if (!p->img_by_fwd) {
            HIPCHK(launch_split_blocks(b.act + b.h_off.back(), b.act_cs, p->ldz, p->N, p->qsplitA, p->qsplitA_cs, C, s));
            HIPCHK(launch_split_blocks(t.act + t.h_off.back(), t.act_cs, p->ldz, p->P, p->qsplitB, p->qsplitB_cs, C, s));
        }
        hipEvent_t stop = nullptr;
        if (int rc = p->timing_begin(VIHMC_T_GRAM, s, &stop)) return rc;
        GramArgs ga = gram_args(p, C);
        ga.aug_done = p->img_by_fwd ? 1 : 0;               // the fused forward wrote feature 100 of both images
        ga.sel = mixed ? 1 : 0;
        ga.bits = resid;
        HIPCHK(launch_gram(ga, s));
        if (stop) HIPCHK(hipEventRecord(stop, s));
        stats_waves = p->gPT * 8;
    }
    if (resid_any || mixed) {
        ContractProb a = side_a(p, C, want_grad, out);
        a.sel = mixed ? 1 : 0;
        a.bits = resid;
        stats_waves_res = p->qchunksA * cdiv(p->P, CONTRACT_OWN_PER_WG) * (a.bf16x6 ? 8 : 4);
        if (a.bf16x6 && !p->img_by_fwd && !gram)
            HIPCHK(launch_split_blocks(a.Q, a.q_cs, a.ldq, p->N, p->qsplitA, p->qsplitA_cs, C, s));
        hipEvent_t stop = nullptr;
        if (int rc = p->timing_begin(VIHMC_T_CONTRACT_A, s, &stop)) return rc;
        HIPCHK(launch_contract(a, C, want_grad, s));
        if (stop) HIPCHK(hipEventRecord(stop, s));
    }
    // gradient evaluations: the statistics run as a slice of the weight-gradient reduce (nothing reads lik or
    // gp slot 0 before the gather)
    StatsJob stats_job{gram ? p->gstats : p->stats, gram ? p->gstats_cs : p->stats_cs, gram ? stats_waves : stats_waves_res,
                       p->lik_buf, p->gp, p->dp, lik_count(p), p->lik.loss, p->lik.tau_out};
    if (mixed) {
        stats_job.stats2 = p->stats;
        stats_job.stats2_cs = p->stats_cs;
        stats_job.n_waves2 = stats_waves_res;
        stats_job.sel = 1;
        stats_job.bits = resid;
    }
    // every chain computed its likelihood: a fit snapshot -- only while the plan runs the Gram form, its one reader (a
    // one-chain plan's device-to-host copy cost ~4 us per evaluation, profiles/r05lt_c1_trace.txt); otherwise the
    // history restarts, so no stale snapshot decides once the form comes on (plan options)
    const bool snap = !gram && guard_live(p) && gram_on(p);
    if (!gram_on(p)) p->n_snap = 0;
    if (snap) {
        // centred: the fit guard compares sum r^2 with sum y~^2 (the Gram form's terms now scale with y~, not y)
        stats_job.fit = p->fit_dev;
        stats_job.ysq = p->gram_center ? p->cysq : p->ysq_dev;
    }
    if (!want_grad) HIPCHK(launch_contract_stats(stats_job, C, s));
    if (want_grad) {
        Net& b = p->nets[0];
        Net& t = p->nets[1];
        if (resid_any || mixed) {
        ContractProb q{};
        q.Own = b.act + b.h_off.back();
        q.own_cs = b.act_cs;
        q.ldown = p->ldz;
        q.Q = t.act + t.h_off.back();
        q.q_cs = t.act_cs;
        q.ldq = p->ldz;
        q.Y = p->gT;           // G^T written by side A: no S recompute on this side
        q.ldy = p->contract_bf16x6 && p->W == 100 ? gt_block_rows(p) : p->ldgT;
        q.y_cs = p->gT_cs;
        q.load_g = 1;
        q.bf16x6 = p->W == 100 ? p->contract_bf16x6 : 0;
        q.qimg = p->qsplitB;
        q.qimg_cs = p->qsplitB_cs;
        q.xcd_group = ((int64_t)C * p->qchunksB) % 8 == 0 ? 1 : 0;
        q.b0 = p->packed;
        q.b0_cs = p->dp;
        q.sel = mixed ? 1 : 0;
        q.bits = resid;
        q.out = p->partB;
        q.out_cs = p->partB_cs;
        q.ldout = p->ldz;
        q.out_chunk_stride = (int64_t)p->N * p->ldz;
        q.stats = p->stats;
        q.Mo = p->N;
        q.Mq = p->P;
        q.W = p->W;
        q.o_tiles = cdiv(p->N, q.bf16x6 ? CONTRACT_BF_B_OWN : CONTRACT_OWN_PER_WG);
        q.q_chunks = p->qchunksB;
        q.q_per_chunk = p->qperB;
        q.with_stats = 0;
        const float v = std::max(p->lik.tau_out, 1e-6f);
        q.gscale = p->lik.loss == VIHMC_LOSS_NLL ? -1.f / v : -p->lik.tau_out;
        if (q.bf16x6 && !p->img_by_fwd)
            HIPCHK(launch_split_blocks(q.Q, q.q_cs, q.ldq, p->P, p->qsplitB, p->qsplitB_cs, C, s));
        hipEvent_t stop = nullptr;
        if (int rc = p->timing_begin(VIHMC_T_CONTRACT_B, s, &stop)) return rc;
        HIPCHK(launch_contract(q, C, true, s));
        if (stop) HIPCHK(hipEventRecord(stop, s));
        const ChainBits* only = mixed ? &resid : nullptr;
        if (p->qchunksA > 1) HIPCHK(launch_reduce(p->jobsA, 2, p->spanA, C, s, nullptr, only));
        else HIPCHK(launch_reduce(p->jobsB, 1, p->spanB, C, s, nullptr, only));
        }

        // diagnostics (plan option debug_dz): the contraction's dZ_b / dZ_t of every chain kept for
        // vihmc_plan_debug_copy("dzb_snap" / "dzt_snap") -- the layer backward overwrites delta[0]
        if (p->debug_dz) {
            if (!p->dzb_snap) {
                if (int rc = p->alloc(&p->dzb_snap, b.delta_cs * p->maxC)) return rc;
                if (int rc = p->alloc(&p->dzt_snap, t.delta_cs * p->maxC)) return rc;
            }
            HIPCHK(hipMemcpyAsync(p->dzb_snap, b.delta[0], sizeof(float) * b.delta_cs * C, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(p->dzt_snap, t.delta[0], sizeof(float) * t.delta_cs * C, hipMemcpyDeviceToDevice, s));
        }
        // backward through both MLPs, last layer first: one fused launch per layer (branch + trunk
        // grouped) computes delta_{l-1} and the dW / db partial slabs
        int cur[2] = {0, 0};
        const int maxl = (int)std::max(b.L.size(), t.L.size());
        // one event pair around the maxl consecutive layer launches (per-launch pairs cost ~4 % of the evaluation):
        // the recorded time includes the maxl - 1 kernel boundaries between them
        hipEvent_t bwd_stop = nullptr;
        if (int rc = p->timing_begin(VIHMC_T_BWD, s, &bwd_stop, maxl)) return rc;
        BwdChainArgs ca{};
        const bool chain = p->bwd_chain && p->bwd_bf16x6 && p->timg_live && bwd_chain_args(p, C, ca);
        if (chain) HIPCHK(launch_bwd_chain(ca, s));
        p->last_bwd_chain = chain;
        for (int i = 0; i < (chain ? 0 : maxl); ++i) {
            BwdArgs ba{};
            ba.C = C;
            int nti = 1;
            for (int net = 0; net < 2; ++net) {
                Net& n = p->nets[net];
                const int j = (int)n.L.size() - 1 - i;
                if (j < 0) continue;
                const LayerPk& L = n.L[j];
                BwdProb& q = ba.p[ba.nprob++];
                q.D = n.delta[cur[net]];
                q.d_cs = n.delta_cs;
                q.ldd = L.ldo;
                q.WT = p->packed + L.wt;
                q.wt_cs = p->dp;
                q.ldw = L.ldo;
                q.H = j == 0 ? n.input : n.act + n.h_off[j - 1];
                q.h_cs = j == 0 ? 0 : n.act_cs;
                q.ldh = L.ldi;
                q.Dout = n.delta[cur[net] ^ 1];
                q.o_cs = n.delta_cs;
                q.part = n.dwpart + L.part_off;
                q.part_cs = n.dwpart_cs;
                q.part_stride = (int32_t)L.part_stride;
                q.M = n.rows;
                q.n_out = L.n_out;
                q.n_in = L.n_in;
                q.act = j >= 1 ? n.L[j - 1].act : 0;
                q.has_dx = j >= 1;
                q.rows_per_wg = L.rows_per_chunk;
                q.n_wg = L.n_chunks;
                nti = std::max(nti, nt_of(L.n_in));
            }
            if (ba.nprob == 1) ba.p[1] = ba.p[0];
            if (p->bwd_bf16x6 && bwd_bf_ok(ba)) HIPCHK(launch_bwd_bf(ba, s));
            else HIPCHK(launch_bwd(ba, nti, s));
            for (int net = 0; net < 2; ++net) {
                const int j = (int)p->nets[net].L.size() - 1 - i;
                if (j >= 1) cur[net] ^= 1;
            }
        }
        if (bwd_stop) HIPCHK(hipEventRecord(bwd_stop, s));
        HIPCHK(launch_reduce(p->bwd_bf16x6 ? p->jobsWt : p->jobsW, p->n_jobsW, p->bwd_bf16x6 ? p->spanWt : p->spanW,
                             C, s, &stats_job));
    }
    HIPCHK(launch_gather_prior(p->gp, p->dp, p->smap_w, theta, p->K, p->prior_mu, p->prior_iv, p->prior_const,
                               p->lik.prior_scale, p->lik_buf, C, logp, want_grad ? grad : nullptr, p->lp_part, p->fin_cnt, s,
                               want_grad ? leap : nullptr));
    if (snap)
        if (int rc = guard_snapshot(p, C, s)) return rc;
    return 0;
}

int mlp_eval(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, float* out, hipStream_t s);

// opt-in (VIHMC_GRAPH=1): measured 0.5-1 % slower than direct launches at C = 1, 4, 16 (the host enqueues an
// evaluation in ~0.06 ms either way, far below its GPU time; the extra theta/logp/grad copies cost more)
bool graphs_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VIHMC_GRAPH");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

int eval_graph(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, hipStream_t s) {
    if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
    if (!p->g_theta) {
        if (int rc = p->alloc(&p->g_theta, (int64_t)p->maxC * p->K)) return rc;
        if (int rc = p->alloc(&p->g_logp, (int64_t)p->maxC)) return rc;
        if (int rc = p->alloc(&p->g_grad, (int64_t)p->maxC * p->K)) return rc;
    }
    hipGraphExec_t exec = nullptr;
    for (auto& g : p->graphs)
        if (g.first == C) exec = g.second;
    if (!exec) {
        if (!p->cap_stream) HIPCHK(hipStreamCreateWithFlags(&p->cap_stream, hipStreamNonBlocking));
        HIPCHK(hipStreamBeginCapture(p->cap_stream, hipStreamCaptureModeThreadLocal));
        p->capturing = true;
        const int rc = p->kind == 0 ? deeponet_eval(p, p->g_theta, C, p->g_logp, p->g_grad, nullptr, p->cap_stream)
                                    : mlp_eval(p, p->g_theta, C, p->g_logp, p->g_grad, nullptr, p->cap_stream);
        p->capturing = false;
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(p->cap_stream, &graph);
        if (rc) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        HIPCHK(ec);
        const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        HIPCHK(ei);
        p->graphs.push_back({C, exec});
    }
    const size_t tb = sizeof(float) * (size_t)C * p->K;
    HIPCHK(hipMemcpyAsync(p->g_theta, theta, tb, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipGraphLaunch(exec, s));
    HIPCHK(hipMemcpyAsync(logp, p->g_logp, sizeof(float) * (size_t)C, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(grad, p->g_grad, tb, hipMemcpyDeviceToDevice, s));
    return 0;
}

int build_mlp(vihmc_plan* p, const vihmc_mlp_desc* d, const float* x, const float* y, const float* frozen,
              const int64_t* idx, const float* prior_mu, const float* prior_sd) {
    if (d->n_layers < 2 || d->n_layers > 6) return fail("MLP plan supports 2..6 linear layers");
    if (d->N < 1 || d->K < 1 || d->max_chains < 1 || d->n_params < 1) return fail("N, K, D, max_chains must be >= 1");
    if (int rc = check_lik(d->lik)) return rc;
    p->kind = 1;
    p->D = d->n_params;
    p->K = d->K;
    p->maxC = d->max_chains;
    p->lik = d->lik;
    MlpArgs& a = p->mlp;
    a.n_layers = d->n_layers;
    a.D = (int32_t)d->n_params;
    a.K = d->K;
    a.N = d->N;
    a.in_dim = d->in_dim;
    a.out_dim = d->out_dim;
    int prev = d->in_dim, maxw = std::max(d->in_dim, d->out_dim);
    std::vector<int> cover(p->D, 0);
    for (int j = 0; j < d->n_layers; ++j) {
        const vihmc_linear& l = d->layers[j];
        if (l.n_in != prev) return fail("layer fan-in does not match the previous fan-out");
        if (l.act < 0 || l.act > 3) return fail("bad activation code");
        a.L[j] = MlpLayer{(int32_t)l.w_off, (int32_t)l.b_off, l.n_out, l.n_in, l.act};
        for (int64_t f = l.w_off; f < l.w_off + (int64_t)l.n_out * l.n_in; ++f) {
            if (f < 0 || f >= p->D) return fail("weight offsets exceed n_params");
            cover[f]++;
        }
        if (l.b_off >= 0)
            for (int64_t f = l.b_off; f < l.b_off + l.n_out; ++f) {
                if (f >= p->D) return fail("bias offsets exceed n_params");
                cover[f]++;
            }
        maxw = std::max(maxw, std::max(l.n_out, l.n_in));
        prev = l.n_out;
    }
    if (prev != d->out_dim) return fail("last layer fan-out != out_dim");
    for (int64_t i = 0; i < p->D; ++i)
        if (cover[i] != 1) return fail("layer table must cover every parameter exactly once");
    if (mlp_lds_bytes((int)p->D, d->n_layers, maxw) > 160 * 1024)
        return fail("MLP plan keeps weights and per-row activations in LDS: D and widths too large for 160 KiB");
    p->maxw = maxw;
    std::vector<int32_t> idx32(p->K);
    for (int k = 0; k < p->K; ++k) {
        if (idx[k] < 0 || idx[k] >= p->D) return fail("sensitive index out of range");
        idx32[k] = (int32_t)idx[k];
    }
    float *dx, *dy, *dfz;
    int32_t* didx;
    if (int rc = p->upload(&dx, x, (int64_t)d->N * d->in_dim)) return rc;
    if (int rc = p->upload(&dy, y, (int64_t)d->N * d->out_dim)) return rc;
    if (int rc = p->upload(&dfz, frozen, p->D)) return rc;
    if (int rc = p->upload(&didx, idx32.data(), p->K)) return rc;
    if (int rc = prior_setup(p, prior_mu, prior_sd)) return rc;
    a.x = dx;
    a.y = dy;
    a.frozen = dfz;
    a.idx = didx;
    a.prior_mu = p->prior_mu;
    a.prior_inv_var = p->prior_iv;
    a.prior_const = p->prior_const;
    a.prior_scale = p->lik.prior_scale;
    a.loss = p->lik.loss;
    a.tau_out = p->lik.tau_out;
    // the reference BNN shape runs on the register-resident kernels (vihmc_bnn.hip): their parameter maps
    a.canon = reinterpret_cast<const int32_t*>(1);   // shape probe only (mlp_bnn_fast_ok reads the table)
    const bool bnn = mlp_bnn_fast_ok(a);
    a.canon = a.cpos = a.goff = nullptr;
    if (bnn) {
        std::vector<int32_t> canon, gpos;
        mlp_bnn_maps(a, canon, gpos);
        std::vector<int32_t> cpos(p->K), goff(p->K);
        for (int k = 0; k < p->K; ++k) {
            cpos[k] = canon[idx32[k]];
            goff[k] = gpos[idx32[k]];
        }
        int32_t *dc, *dcp, *dgo;
        if (int rc = p->upload(&dc, canon.data(), p->D)) return rc;
        if (int rc = p->upload(&dcp, cpos.data(), p->K)) return rc;
        if (int rc = p->upload(&dgo, goff.data(), p->K)) return rc;
        a.canon = dc;
        a.cpos = dcp;
        a.goff = dgo;
    }
    return 0;
}

int mlp_eval(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, float* out, hipStream_t s) {
    if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
    MlpArgs a = p->mlp;
    a.theta = theta;
    a.logp = logp;
    a.grad = grad;
    a.out = out;
    hipEvent_t stop = nullptr;
    if (int rc = p->timing_begin(VIHMC_T_MLP, s, &stop)) return rc;
    if (p->mlp_fast && mlp_bnn_fast_ok(a)) HIPCHK(launch_mlp_bnn(a, C, s));
    else HIPCHK(launch_mlp(a, C, p->maxw, s));
    if (stop) HIPCHK(hipEventRecord(stop, s));
    return 0;
}

template <typename F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::exception& e) {
        return fail(std::string("exception: ") + e.what());
    } catch (...) {
        return fail("unknown exception");
    }
}

}  // namespace

extern "C" {

int vihmc_deeponet_plan_create(vihmc_plan** out, const vihmc_deeponet_desc* d, const float* x_branch,
                               const float* trunk_feat, const float* y, const float* frozen, const int64_t* sens_idx,
                               const float* prior_mu, const float* prior_sd, int device) {
    return guarded([&]() -> int {
        if (!out || !d || !x_branch || !trunk_feat || !y || !frozen || !sens_idx || !prior_mu || !prior_sd)
            return fail("null argument");
        *out = nullptr;
        HIPCHK(hipSetDevice(device));
        auto* p = new vihmc_plan();
        p->device = device;
        if (int rc = build_deeponet(p, d, x_branch, trunk_feat, y, frozen, sens_idx, prior_mu, prior_sd)) {
            delete p;
            return rc;
        }
        *out = p;
        return 0;
    });
}

int vihmc_mlp_plan_create(vihmc_plan** out, const vihmc_mlp_desc* d, const float* x, const float* y,
                          const float* frozen, const int64_t* sens_idx, const float* prior_mu, const float* prior_sd,
                          int device) {
    return guarded([&]() -> int {
        if (!out || !d || !x || !y || !frozen || !sens_idx || !prior_mu || !prior_sd || !d->layers)
            return fail("null argument");
        *out = nullptr;
        HIPCHK(hipSetDevice(device));
        auto* p = new vihmc_plan();
        p->device = device;
        if (int rc = build_mlp(p, d, x, y, frozen, sens_idx, prior_mu, prior_sd)) {
            delete p;
            return rc;
        }
        *out = p;
        return 0;
    });
}

int vihmc_logp_grad(vihmc_plan* p, const float* theta, int C, float* logp, float* grad, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta || !logp) return fail("null argument");
        hipStream_t s = static_cast<hipStream_t>(stream);
        const bool g_on = p->graph_on < 0 ? graphs_enabled() : p->graph_on != 0;
        if (grad && !p->timing_on && g_on) return eval_graph(p, theta, C, logp, grad, s);
        return p->kind == 0 ? deeponet_eval(p, theta, C, logp, grad, nullptr, s)
                            : mlp_eval(p, theta, C, logp, grad, nullptr, s);
    });
}

int vihmc_grad(vihmc_plan* p, const float* theta, int C, float* grad, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta || !grad) return fail("null argument");
        hipStream_t s = static_cast<hipStream_t>(stream);
        if (p->kind == 0) return deeponet_eval(p, theta, C, nullptr, grad, nullptr, s);
        if (!p->lik_buf)                                  // BNN plans: the value lands in a plan-owned scratch
            if (int rc = p->alloc(&p->lik_buf, p->maxC)) return rc;
        if (int rc = mlp_eval(p, theta, C, p->lik_buf, grad, nullptr, s)) return rc;
        return 0;
    });
}

int vihmc_split_step(vihmc_plan* p, float* theta, float* momentum, int C, float* grad, float* logp, int mode, float kick,
                     float drift, vihmc_plan* scatter_into, int scattered_in, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta || !momentum || !grad) return fail("null argument");
        if (p->kind != 0) return fail("vihmc_split_step needs a DeepONet plan");
        if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
        if (mode != 1 && mode != 2) return fail("vihmc_split_step: mode must be 1 or 2");
        if (scatter_into && (scatter_into->kind != 0 || scatter_into->dp != p->dp || scatter_into->K != p->K ||
                             scatter_into->maxC < C))
            return fail("vihmc_split_step: scatter_into must be a DeepONet plan of the same layout");
        hipStream_t s = static_cast<hipStream_t>(stream);
        LeapArgs lf{};
        lf.p = momentum;
        lf.th = theta;
        lf.mode = mode;
        lf.kick = kick;
        lf.drift = drift;
        // plan option fuse_scatter = 0 (the A/B path, as in vihmc_trajectory): such a plan receives no scatter from
        // the previous shard's gather and runs its own k_scatter, whatever the caller says
        lf.scattered_in = scattered_in && p->fuse_scatter ? 1 : 0;
        if (mode == 1 && scatter_into && scatter_into->fuse_scatter) {
            vihmc_plan* q = scatter_into;
            const ScatterImg si = scatter_img(q);
            lf.sc = ScatterArgs{q->packed, q->dp, q->smap_w, q->smap_wt, q->img_by_scatter ? si : ScatterImg{}};
        }
        return deeponet_eval(p, theta, C, logp, grad, nullptr, s, &lf);
    });
}

int vihmc_mlp_trajectory(vihmc_plan* p, const float* theta_in, float* theta_out, const float* p_in, float* p_out,
                         const float* g_in, float* g_out, float* logp_out, const float* eps, const float* inv_mass,
                         int L, int C, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta_in || !theta_out || !p_in || !p_out || !g_in || !g_out || !logp_out || !eps)
            return fail("null argument");
        if (p->kind != 1) return fail("vihmc_mlp_trajectory needs a BNN (MLP) plan");
        if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
        if (L < 1) return fail("L must be >= 1");
        if (theta_in == theta_out) return fail("theta_out must not alias theta_in (the sampler reverts to it)");
        hipStream_t s = static_cast<hipStream_t>(stream);
        MlpTrajArgs t{theta_in, theta_out, p_in, p_out, g_in, g_out, logp_out, eps, inv_mass, L, 0};
        hipEvent_t stop = nullptr;
        if (int rc = p->timing_begin(VIHMC_T_MLP, s, &stop, L)) return rc;
        if (p->mlp_fast && mlp_bnn_fast_ok(p->mlp)) HIPCHK(launch_mlp_traj_bnn(p->mlp, t, C, s));
        else HIPCHK(launch_mlp_traj(p->mlp, t, C, p->maxw, s));
        if (stop) HIPCHK(hipEventRecord(stop, s));
        return 0;
    });
}

int vihmc_trajectory(vihmc_plan* p, const float* theta_in, float* theta_out, const float* p_in, float* p_out,
                     const float* g_in, float* g_out, float* logp_out, const float* eps, const float* inv_mass, int L,
                     int C, void* stream) {
    if (p && p->kind == 1)
        return vihmc_mlp_trajectory(p, theta_in, theta_out, p_in, p_out, g_in, g_out, logp_out, eps, inv_mass, L, C,
                                    stream);
    return guarded([&]() -> int {
        if (!p || !theta_in || !theta_out || !p_in || !p_out || !g_in || !g_out || !logp_out || !eps)
            return fail("null argument");
        if (C < 1 || C > p->maxC) return fail("C must be in [1, max_chains]");
        if (L < 1) return fail("L must be >= 1");
        if (theta_in == theta_out) return fail("theta_out must not alias theta_in (the sampler reverts to it)");
        if (p_in == p_out) return fail("p_out must not alias p_in");
        hipStream_t s = static_cast<hipStream_t>(stream);
        // opening half step + first position step, then L evaluations whose gradient gather applies the
        // momentum step and the next position step in place (theta_out / p_out are the running state)
        // every new position is scattered into the packed weights / images by the kernel that computes it (the opening
        // kernel, then each step's gradient gather), so the evaluations skip their k_scatter (VIHMC_FUSE_SCATTER=0:
        // the evaluations scatter as usual)
        const bool fuse = p->fuse_scatter != 0;
        const ScatterImg si = scatter_img(p);
        const ScatterArgs sc{p->packed, p->dp, p->smap_w, p->smap_wt, p->img_by_scatter ? si : ScatterImg{}};
        HIPCHK(launch_leap_open(theta_in, theta_out, p_in, p_out, g_in, eps, inv_mass, p->K, C, s, fuse ? &sc : nullptr));
        for (int st = 0; st < L; ++st) {
            LeapArgs lf{p_out, theta_out, eps, inv_mass, st == L - 1 ? 1 : 0, fuse && st < L - 1 ? sc : ScatterArgs{},
                        fuse ? 1 : 0};
            // only the end point's log-prob is returned: the intermediate evaluations skip the log-prob finalisation
            if (int rc = deeponet_eval(p, theta_out, C, st == L - 1 ? logp_out : nullptr, g_out, nullptr, s, &lf))
                return rc;
        }
        return 0;
    });
}

int vihmc_kinetic_slices(int K) { return K >= 1 ? kinetic_slices(K) : -1; }

int vihmc_kinetic(const float* p, const float* inv_mass, int C, int K, float* ke, double* part, uint32_t* cnt,
                  void* stream) {
    return guarded([&]() -> int {
        if (C < 1 || K < 1) return fail("vihmc_kinetic: C, K >= 1");
        if (!p || !ke || !part || !cnt) return fail("null argument");
        HIPCHK(launch_kinetic(p, inv_mass, C, K, ke, part, cnt, static_cast<hipStream_t>(stream)));
        return 0;
    });
}

int vihmc_hmc_accept(int C, int K, int n, int burn, const float* lp0, const float* lp1, const float* ke0,
                     const float* ke1, const float* logu, const float* th1, const float* g1,
                     float* th_last, float* lp_last, float* g_last, float* th_bp, float* lp_bp, float* g_bp,
                     float* th_cur, float* lp_cur, float* g_cur, float* samples, int64_t s_cap, int64_t* counts,
                     uint8_t* accepted, int64_t acc_ld, float* trace, int64_t tr_ld, float* rho, uint8_t* err,
                     void* stream) {
    return guarded([&]() -> int {
        if (C < 1 || K < 1 || n < 0) return fail("vihmc_hmc_accept: C, K >= 1, n >= 0");
        if (!lp0 || !lp1 || !ke0 || !ke1 || !logu || !th1 || !g1 || !th_last || !lp_last || !g_last || !accepted ||
            !trace || !rho || !err)
            return fail("null argument");
        if (burn && (!th_bp || !lp_bp || !g_bp || !th_cur || !lp_cur || !g_cur))
            return fail("vihmc_hmc_accept: burn-in needs the fallback and current-state buffers");
        if (!burn && samples && (!counts || s_cap < 2)) return fail("vihmc_hmc_accept: samples need counts, s_cap >= 2");
        if (n >= acc_ld || n >= tr_ld) return fail("vihmc_hmc_accept: n outside the accepted / trace rows");
        AcceptArgs a{};
        a.K = K;
        a.n = n;
        a.burn = burn ? 1 : 0;
        a.lp0 = lp0;
        a.lp1 = lp1;
        a.ke0 = ke0;
        a.ke1 = ke1;
        a.logu = logu;
        a.th1 = th1;
        a.g1 = g1;
        a.th_last = th_last;
        a.lp_last = lp_last;
        a.g_last = g_last;
        a.th_bp = th_bp;
        a.lp_bp = lp_bp;
        a.g_bp = g_bp;
        a.th_cur = th_cur;
        a.lp_cur = lp_cur;
        a.g_cur = g_cur;
        a.samples = burn ? nullptr : samples;
        a.s_cap = s_cap;
        a.counts = counts;
        a.accepted = accepted;
        a.acc_ld = acc_ld;
        a.trace = trace;
        a.tr_ld = tr_ld;
        a.rho = rho;
        a.err = err;
        HIPCHK(launch_hmc_accept(a, C, static_cast<hipStream_t>(stream)));
        return 0;
    });
}

int vihmc_forward(vihmc_plan* p, const float* theta, int C, float* logp, float* out, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta || !logp || !out) return fail("null argument");
        hipStream_t s = static_cast<hipStream_t>(stream);
        return p->kind == 0 ? deeponet_eval(p, theta, C, logp, nullptr, out, s)
                            : mlp_eval(p, theta, C, logp, nullptr, out, s);
    });
}

namespace {
int ld_residue(int n, int res) {       // smallest v >= n with v % 16 == res
    int v = n;
    while (v % 16 != res) ++v;
    return v;
}

// DeepONet sensitivity (vihmc_sens.hip): pair tasks built on the host from the point lists, one forward
// of chain 0, then seeds -> outer -> reduce -> flat. Temporaries are freed after a stream sync.
int deeponet_sensitivity(vihmc_plan* p, const float* theta, const int32_t* pts, int npts, const float* sigma,
                         float* out, hipStream_t s) {
    if (!pts || npts < 1) return fail("DeepONet sensitivity needs point lists (pts, npts >= 1)");
    const int N = p->N, P = p->P;
    for (int64_t e = 0; e < (int64_t)N * npts; ++e)
        if (pts[e] < 0 || pts[e] >= P) return fail("point index out of range [0, P)");
    for (int net = 0; net < 2; ++net)
        if ((int)p->nets[net].L.size() > SENS_MAXL) return fail("sensitivity: too many layers");
    // branch: group n, seeds = trunk rows pts[n][*]; trunk: group p, seeds = branch rows n with p in pts[n]
    std::vector<int32_t> tasks[2], seeds[2];
    seeds[0].assign(pts, pts + (int64_t)N * npts);
    for (int n = 0; n < N; ++n)
        for (int k = 0; k < npts; k += SENS_SEEDS)
            tasks[0].insert(tasks[0].end(), {n, n * npts + k, std::min(SENS_SEEDS, npts - k)});
    {
        std::vector<int32_t> cnt(P + 1, 0);
        for (int64_t e = 0; e < (int64_t)N * npts; ++e) ++cnt[pts[e] + 1];
        for (int q = 0; q < P; ++q) cnt[q + 1] += cnt[q];
        std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
        seeds[1].resize((size_t)N * npts);
        for (int n = 0; n < N; ++n)
            for (int k = 0; k < npts; ++k) seeds[1][fill[pts[(int64_t)n * npts + k]]++] = n;
        for (int q = 0; q < P; ++q)
            for (int k = cnt[q]; k < cnt[q + 1]; k += SENS_SEEDS)
                tasks[1].insert(tasks[1].end(), {q, k, std::min(SENS_SEEDS, cnt[q + 1] - k)});
    }
    std::vector<void*> tmp;
    auto talloc = [&](void** d, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(d, std::max<size_t>(bytes, 4));
        if (e == hipSuccess) tmp.push_back(*d);
        return e;
    };
    auto cleanup = [&]() {
        (void)hipStreamSynchronize(s);
        for (void* v : tmp) (void)hipFree(v);
    };
    SensArgs a{};
    int kmax = 16, jmax = 16;
    hipError_t e = hipSuccess;
    for (int net = 0; net < 2 && e == hipSuccess; ++net) {
        Net& n = p->nets[net];
        Net& o = p->nets[1 - net];
        SensNet& sn = a.net[net];
        sn.nl = (int)n.L.size();
        sn.n_tasks = (int)(tasks[net].size() / 3);
        sn.n_wg = cdiv(sn.n_tasks, SENS_WAVES);
        sn.chunks = std::max(1, std::min(128, cdiv(sn.n_tasks, 256)));
        sn.tasks_per_chunk = cdiv(sn.n_tasks, sn.chunks);
        sn.seeds = o.act + o.h_off.back();
        sn.ld_seed = p->ldz;
        for (int l = 0; l < sn.nl; ++l) {
            const LayerPk& L = n.L[l];
            SensLayer& q = sn.L[l];
            q.W = p->packed + L.wp;
            q.wp = L.wp;
            q.bias = L.bias;
            q.ldi = L.ldi;
            q.n_out = L.n_out;
            q.n_in = L.n_in;
            q.Hprev = l == 0 ? n.input : n.act + n.h_off[l - 1];
            q.ldh = l == 0 ? n.ld_in : n.L[l - 1].ldo;
            q.act_prev = l == 0 ? ACT_ID : n.L[l - 1].act;
            kmax = std::max(kmax, (L.n_out + 15) & ~15);
            jmax = std::max(jmax, (L.n_in + 15) & ~15);
        }
        int32_t *dt = nullptr, *ds = nullptr;
        e = talloc((void**)&dt, tasks[net].size() * 4);
        if (e == hipSuccess) e = talloc((void**)&ds, seeds[net].size() * 4);
        if (e == hipSuccess) e = hipMemcpyAsync(dt, tasks[net].data(), tasks[net].size() * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(ds, seeds[net].data(), seeds[net].size() * 4, hipMemcpyHostToDevice, s);
        sn.tasks = dt;
        sn.seed_idx = ds;
        if (e == hipSuccess) e = talloc((void**)&sn.Q, (size_t)std::max(sn.n_tasks, 1) * sn.nl * SENS_QLD * 4);
        if (e == hipSuccess) e = hipMemsetAsync(sn.Q, 0, (size_t)std::max(sn.n_tasks, 1) * sn.nl * SENS_QLD * 4, s);
        if (e == hipSuccess) e = talloc((void**)&sn.part, (size_t)sn.nl * sn.chunks * SENS_PART * 4);
    }
    int32_t* dmap = nullptr;
    if (e == hipSuccess) e = talloc((void**)&a.S, (size_t)p->dp * 4);
    if (e == hipSuccess) e = hipMemsetAsync(a.S, 0, (size_t)p->dp * 4, s);
    if (e == hipSuccess) e = talloc((void**)&dmap, (size_t)p->D * 4);
    if (e == hipSuccess) e = hipMemcpyAsync(dmap, p->fmap_host.data(), (size_t)p->D * 4, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
        cleanup();
        return fail(std::string("sensitivity setup: ") + hipGetErrorString(e), (int)e);
    }
    (void)kmax;
    (void)jmax;
    a.ldd = ld_residue(128, 8);       // deltas [16][136]: float4 row reads of 16 rows are conflict free
    a.ldw = ld_residue(128, 4);       // W image [128][132]: b32 reads of rows 4 apart hit distinct bank groups
    a.count = (float)((double)N * npts);
    const ScatterImg si = scatter_img(p);
    e = launch_scatter(p->packed, p->dp, 1, theta, p->K, p->smap_w, p->smap_wt, s, p->img_by_scatter ? &si : nullptr);
    int rc = e == hipSuccess ? deeponet_forward_layers(p, 1, s, false, false) : 0;
    SensArgs* dev_a = nullptr;
    if (e == hipSuccess && rc == 0) e = talloc((void**)&dev_a, sizeof(SensArgs));
    if (e == hipSuccess && rc == 0) e = hipMemcpyAsync(dev_a, &a, sizeof(SensArgs), hipMemcpyHostToDevice, s);
    if (e == hipSuccess && rc == 0) e = launch_sens(a, dev_a, dmap, p->D, sigma, out, s);
    cleanup();
    if (rc) return rc;
    if (e != hipSuccess) return fail(std::string("sensitivity: ") + hipGetErrorString(e), (int)e);
    return 0;
}

int mlp_sensitivity(vihmc_plan* p, const float* theta, const float* sigma, float* out, hipStream_t s) {
    MlpArgs a = p->mlp;
    a.theta = theta;
    float* slab = nullptr;
    const int nblk = cdiv(p->mlp.N, 64);
    HIPCHK(hipMalloc((void**)&slab, (size_t)nblk * p->D * 4));
    hipError_t e = launch_sens_mlp(a, slab, sigma, out, p->maxw, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(slab);
    if (e != hipSuccess) return fail(std::string("sensitivity (MLP): ") + hipGetErrorString(e), (int)e);
    return 0;
}
}  // namespace

int vihmc_sensitivity(vihmc_plan* p, const float* theta, const int32_t* pts, int npts, const float* sigma,
                      float* out, void* stream) {
    return guarded([&]() -> int {
        if (!p || !theta || !out) return fail("null argument");
        hipStream_t s = static_cast<hipStream_t>(stream);
        return p->kind == 0 ? deeponet_sensitivity(p, theta, pts, npts, sigma, out, s)
                            : mlp_sensitivity(p, theta, sigma, out, s);
    });
}

int vihmc_plan_set_data(vihmc_plan* p, const float* x_branch, const float* y, void* stream) {
    return guarded([&]() -> int {
        if (!p || !x_branch || !y) return fail("null argument");
        if (p->kind != 0) return fail("vihmc_plan_set_data: DeepONet plans only");
        hipStream_t s = static_cast<hipStream_t>(stream);
        Net& b = p->nets[0];
        const size_t in_b = (size_t)b.L[0].n_in * sizeof(float);
        // branch rows into the padded [N][ld_in] input (pad columns stay zero), y as is
        HIPCHK(hipMemcpy2DAsync(b.input, (size_t)b.ld_in * sizeof(float), x_branch, in_b, in_b, (size_t)b.rows,
                                hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(p->y, y, (size_t)p->N * p->P * sizeof(float), hipMemcpyDeviceToDevice, s));
        return gram_images(p, s);
    });
}

int vihmc_plan_set_trunk_rows(vihmc_plan* p, const float* trunk_all, const float* y_all, int64_t P_all,
                              const int32_t* ind, void* stream) {
    return guarded([&]() -> int {
        if (!p || !trunk_all || !y_all || !ind) return fail("null argument");
        if (p->kind != 0) return fail("vihmc_plan_set_trunk_rows: DeepONet plans only");
        if (P_all < p->P) return fail("vihmc_plan_set_trunk_rows: P_all smaller than the plan's P");
        Net& t = p->nets[1];
        HIPCHK(launch_gather_trunk(trunk_all, t.L[0].n_in, y_all, P_all, ind, p->P, p->N, t.input, t.ld_in, p->y,
                                   static_cast<hipStream_t>(stream)));
        return gram_images(p, static_cast<hipStream_t>(stream));
    });
}

int vihmc_plan_kind(const vihmc_plan* p) { return p ? p->kind : -1; }
int64_t vihmc_plan_n_params(const vihmc_plan* p) { return p ? p->D : -1; }
int vihmc_plan_K(const vihmc_plan* p) { return p ? p->K : -1; }
int vihmc_plan_max_chains(const vihmc_plan* p) { return p ? p->maxC : -1; }
int64_t vihmc_plan_device_bytes(const vihmc_plan* p) { return p ? p->bytes : -1; }

int vihmc_timing_enable(vihmc_plan* p, int which, int on) {
    if (!p) return fail("null plan");
    if (which < -1 || which >= VIHMC_T_COUNT) return fail("timing class out of range");
    const int bits = which < 0 ? (1 << VIHMC_T_COUNT) - 1 : 1 << which;
    p->timing_on = on ? (p->timing_on | bits) : (p->timing_on & ~bits);
    p->ev_used = 0;
    p->ev_cls.clear();
    p->ev_nl.clear();
    return 0;
}

int vihmc_timing_read_class(vihmc_plan* p, int which, double* total_ms, int64_t* launches) {
    if (!p || !total_ms || !launches) return fail("null argument");
    double t = 0.0;
    int64_t n = 0;
    for (size_t i = 0; i + 1 < p->ev_used; i += 2) {
        if (which >= 0 && p->ev_cls[i / 2] != which) continue;
        HIPCHK(hipEventSynchronize(p->ev_pool[i + 1]));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, p->ev_pool[i], p->ev_pool[i + 1]));
        t += ms;
        n += p->ev_nl[i / 2];
    }
    *total_ms = t;
    *launches = n;
    return 0;
}

int vihmc_timing_read(vihmc_plan* p, double* total_ms, int64_t* launches) {
    const int rc = vihmc_timing_read_class(p, -1, total_ms, launches);
    if (p && rc == 0) {
        p->ev_used = 0;
        p->ev_cls.clear();
    }
    return rc;
}

int vihmc_timing_reset(vihmc_plan* p) {
    if (!p) return fail("null plan");
    p->ev_used = 0;
    p->ev_cls.clear();
    return 0;
}

#define OPTION_KEYS "fwd_bf16x6, contract_bf16x6, bwd_bf16x6, graph, timing_every, fwd_wimg, fwd_in0, skip_zt, fuse_scatter, img_scatter, mlp_fast, bwd_chain, gram, gram_active, gram_center, gram_pair2, tanh_cr, debug_dz, gram_min_chains, gram_guard, grad_evals, gram_evals, gram_chains, gram_chain_evals, y_masked, lik_count"

int vihmc_plan_option(vihmc_plan* p, const char* key, int value) {
    if (!p || !key) return fail("null argument");
    const std::string k(key);
    if (k == "fwd_bf16x6") p->fwd_bf16x6 = value ? 1 : 0;
    else if (k == "contract_bf16x6") p->contract_bf16x6 = value ? 1 : 0;
    else if (k == "bwd_bf16x6") p->bwd_bf16x6 = value ? 1 : 0;
    else if (k == "graph") p->graph_on = value ? 1 : 0;
    else if (k == "fwd_wimg") p->fwd_wimg = value ? 1 : 0;
    else if (k == "fwd_in0") p->fwd_in0 = value ? 1 : 0;
    else if (k == "skip_zt") p->skip_zt = value ? 1 : 0;
    else if (k == "timing_every") {
        p->timing_every = std::max(1, value);
        return 0;                                               // not a kernel choice: graphs stay
    }
    else if (k == "fuse_scatter") p->fuse_scatter = value ? 1 : 0;
    else if (k == "img_scatter") p->img_by_scatter = value && p->smap_img;   // 0: split the images per evaluation
    else if (k == "mlp_fast") p->mlp_fast = value ? 1 : 0;
    else if (k == "bwd_chain") p->bwd_chain = value ? 1 : 0;
    else if (k == "gram") p->gram = value ? 1 : 0;
    else if (k == "gram_min_chains") p->gram_min_chains = std::max(1, value);
    else if (k == "gram_guard") {                               // threshold 10^-value (0: off); history restarts
        p->gram_guard = std::max(0, value);
        p->n_snap = 0;
    }
    else if (k == "y_masked" || k == "lik_count") {             // per-item target subsets (VI training, p < P)
        if (p->kind != 0) return fail("plan option '" + k + "': DeepONet plans only");
        if (k == "y_masked") p->y_masked = value ? 1 : 0;
        else if (value < 0 || (double)value > (double)p->N * (double)p->P) return fail("lik_count must be in [0, N P]");
        else p->lik_count = value;
    }
    else if (k == "gram_active") return fail("plan option 'gram_active' is read-only");
    else if (k == "debug_dz") {
        p->debug_dz = value ? 1 : 0;
        return 0;
    }
    else if (k == "tanh_cr") {                                  // forward: the centre (a forward output) is stale
        p->tanh_cr = value ? 1 : 0;
        p->centre_stale = true;
    }
    else if (k == "gram_pair2") {                               // two-chain T_t units (bitwise the same dZt);
        if (value < 0 || value > 2) return fail("gram_pair2: 0, 1 or 2");
        p->gram_pair2 = value;                                  // 2: on every row group (tests)
    }
    else if (k == "gram_center") {                              // centred Gram form (1) or y itself (0)
        if ((value ? 1 : 0) != p->gram_center) {
            p->gram_center = value ? 1 : 0;
            if (int rc = gram_images(p, nullptr)) return rc;    // y images now, or the centre at the next evaluation
            HIPCHK(hipDeviceSynchronize());
        }
    }
    else if (k == "grad_evals" || k == "gram_evals") {          // counters: any value resets both
        p->n_grad_calls = p->n_gram_calls = p->n_gram_chain_evals = 0;
        return 0;
    }
    else return fail("unknown plan option '" + k + "' (" OPTION_KEYS ")");
    // captured graphs embed the kernel choice
    for (auto& g : p->graphs) (void)hipGraphExecDestroy(g.second);
    p->graphs.clear();
    return 0;
}

int vihmc_plan_get_option(const vihmc_plan* p, const char* key, int* value) {
    if (!p || !key || !value) return fail("null argument");
    const std::string k(key);
    if (k == "fwd_bf16x6") *value = p->fwd_bf16x6;
    else if (k == "contract_bf16x6") *value = p->contract_bf16x6 && p->W == 100;
    else if (k == "bwd_bf16x6") *value = p->bwd_bf16x6;
    else if (k == "graph") *value = p->graph_on;
    else if (k == "fwd_wimg") *value = p->fwd_wimg;
    else if (k == "fwd_in0") *value = p->kind == 0 && fused_forward_ok(p) && fused_input_ok(p);
    else if (k == "skip_zt") *value = p->skip_zt;
    else if (k == "timing_every") *value = p->timing_every;
    else if (k == "fuse_scatter") *value = p->fuse_scatter;
    else if (k == "img_scatter") *value = p->img_by_scatter ? 1 : 0;
    else if (k == "mlp_fast") *value = p->mlp_fast && p->kind == 1 && mlp_bnn_fast_ok(p->mlp);
    else if (k == "bwd_chain") *value = p->bwd_chain | (p->last_bwd_chain ? 2 : 0);
    else if (k == "gram") *value = (p->gram && p->gram_alloc ? 1 : 0) | (p->last_gram ? 2 : 0);
    else if (k == "gram_min_chains") *value = p->gram_min_chains;
    // whether this plan's gradient-only evaluations can take the Gram form at all (gram, width, max_chains >=
    // gram_min_chains, no target mask, and a plan beyond GUARD_MAXC chains only with the fit guard off): a plan that
    // falls back to the residual form for its chain count says so here
    else if (k == "gram_active") *value = gram_on(p) ? 1 : 0;
    else if (k == "gram_center") *value = p->gram_center;
    else if (k == "gram_pair2") *value = p->gram_pair2;
    else if (k == "tanh_cr") *value = p->tanh_cr;
    else if (k == "debug_dz") *value = p->debug_dz;
    else if (k == "grad_evals") *value = (int)std::min<int64_t>(p->n_grad_calls, INT32_MAX);
    else if (k == "gram_evals") *value = (int)std::min<int64_t>(p->n_gram_calls, INT32_MAX);
    else if (k == "gram_chains") *value = p->last_gram_chains;
    else if (k == "gram_chain_evals") *value = (int)std::min<int64_t>(p->n_gram_chain_evals, INT32_MAX);
    else if (k == "gram_guard") *value = p->gram_guard;
    else if (k == "y_masked") *value = p->y_masked;
    else if (k == "lik_count") *value = (int)std::min<double>(lik_count(p), INT32_MAX);
    else return fail("unknown plan option '" + k + "' (" OPTION_KEYS ")");
    return 0;
}

int vihmc_plan_check_canaries(vihmc_plan* p, int64_t* corrupted) {
    return guarded([&]() -> int {
        if (!p || !corrupted) return fail("null argument");
        if (!p->canary) return fail("vihmc_plan_check_canaries: plan created without VIHMC_CANARY=1");
        HIPCHK(hipDeviceSynchronize());
        std::vector<unsigned char> h(CANARY_BYTES);
        int64_t bad = 0;
        for (unsigned char* c : p->canaries) {
            HIPCHK(hipMemcpy(h.data(), c, CANARY_BYTES, hipMemcpyDeviceToHost));
            for (unsigned char v : h) bad += v != 0xA5;
        }
        *corrupted = bad;
        return 0;
    });
}

// diagnostics: copy one internal buffer (all chains) to host memory; dst == null returns its size in *bytes
int vihmc_plan_debug_copy(vihmc_plan* p, const char* name, void* dst, int64_t* bytes) {
    return guarded([&]() -> int {
        if (!p || !name || !bytes) return fail("null argument");
        if (p->kind != 0) return fail("vihmc_plan_debug_copy: DeepONet plans only");
        const std::string k(name);
        const void* src = nullptr;
        int64_t n = 0;
        const Net& b = p->nets[0];
        const Net& t = p->nets[1];
        const int64_t C = p->maxC;
        if (k == "dzb") src = b.delta[0], n = 4 * b.delta_cs * C;
        else if (k == "dzt") src = t.delta[0], n = 4 * t.delta_cs * C;
        else if (k == "act_b") src = b.act, n = 4 * b.act_cs * C;
        else if (k == "act_t") src = t.act, n = 4 * t.act_cs * C;
        else if (k == "bimg") src = p->qsplitA, n = p->qsplitA_cs * C;
        else if (k == "timg") src = p->qsplitB, n = p->qsplitB_cs * C;
        else if (k == "gram_tb") src = p->gtb_part, n = 4 * p->gtb_cs * C;
        else if (k == "gram_gt_part") src = p->ggt_part, n = 8 * p->ggt_part_cs * C;
        else if (k == "gram_gb_part") src = p->ggb_part, n = 8 * p->ggb_part_cs * C;
        else if (k == "gram_tb_sum") src = p->gtb_sum, n = 4 * p->gtbs_cs * C;
        else if (k == "gram_gt") src = p->ggt, n = 4 * 112 * 112 * C;
        else if (k == "gram_gt64") src = p->ggt64, n = 8 * 112 * 112 * C;
        else if (k == "gram_gb3") src = p->ggb3, n = 4 * (int64_t)GRAM_P3_BLOCK * C;
        else if (k == "gram_gb") src = p->ggb, n = 4 * (int64_t)CONTRACT_SPLIT_BLOCK * C;
        else if (k == "gram_tt") src = p->gtt_part, n = 4 * p->gtt_cs * C;
        else if (k == "gram_stats") src = p->gstats, n = 8 * p->gstats_cs * C;
        else if (k == "gram_ht") src = p->ght, n = 4 * 112 * 112 * C;
        else if (k == "dzb_snap") src = p->dzb_snap, n = 4 * b.delta_cs * C;
        else if (k == "dzt_snap") src = p->dzt_snap, n = 4 * t.delta_cs * C;
        else if (k == "gram_ht_part") src = p->ght_part, n = 4 * p->ght_cs * C;
        else if (k == "gram_hb_part") src = p->ghb_part, n = 4 * p->ghb_cs * C;
        else if (k == "gram_gcol") src = p->gcol, n = 8 * 4 * 112 * C;
        else if (k == "center_bimg") src = p->cimgB, n = p->cimgB ? p->qsplitA_cs : 0;
        else if (k == "center_timg") src = p->cimgT, n = p->cimgT ? p->qsplitB_cs : 0;
        else if (k == "center_b0") src = p->cB0, n = p->cB0 ? 4 * (int64_t)p->N * p->ldz : 0;
        else if (k == "center_col") src = p->ccol, n = p->ccol ? 8 * 112 : 0;
        else if (k == "center_ysq") src = p->cysq, n = p->cysq ? 16 : 0;
        else return fail("vihmc_plan_debug_copy: unknown buffer " + k);
        if (!src) n = 0;
        *bytes = n;
        if (!dst || !n) return 0;
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(dst, src, (size_t)n, hipMemcpyDeviceToHost));
        return 0;
    });
}

int vihmc_clock_stamp(uint64_t* out, void* stream) {
    return guarded([&]() -> int {
        if (!out) return fail("null argument");
        HIPCHK(launch_clock_stamp(reinterpret_cast<unsigned long long*>(out), static_cast<hipStream_t>(stream)));
        return 0;
    });
}

int vihmc_graph_enable(vihmc_plan* p, int on) {
    if (!p) return fail("null plan");
    p->graph_on = on ? 1 : 0;
    return 0;
}

void vihmc_plan_destroy(vihmc_plan* p) { delete p; }
const char* vihmc_last_error(void) { return g_err.c_str(); }
const char* vihmc_version(void) {
    static std::string v = "vihmc 0.3.0 gfx950 diag=" + std::to_string(vihmc::diag_switches());
    return v.c_str();
}

}  // extern "C"
