// 1x1-convolution GEMMs with the conv epilogue fused (hipBLASLt).
//
// On channels_last (NHWC) tensors a stride-1 1x1 convolution is the GEMM
//   D[M][N] = A[M][K] . W[N][K]^T,  M = batch*H*W, K = Cin, N = Cout,
// and the reference's frozen-BN bottleneck tail (ResNet.py:246-294
// bottleneck_transformation: conv3 -> AffineChannel -> + residual -> ReLU, the
// AffineChannel folded into W and bias) is
//   D = relu(A . W^T + bias + R)
// which hipBLASLt computes in ONE kernel: alpha*op(A)op(B) + beta*C with the
// bias + ReLU epilogue, C = the residual.  That replaces MIOpen's conv output
// write + vd_bias_act's read of it, read of the residual and write of the sum
// (4 tensor passes) with the residual read and one write (2 passes).
//
// hipBLASLt is column-major: the row-major problem is issued as
//   D'(N x M) = op_T(W stored K x N) . A'(K x M) + beta C'(N x M) + bias(N)
// where X' is the column-major view of row-major X (no data movement).
// Algorithms: hipblasLtMatmulAlgoGetHeuristic's top kMaxAlgos candidates per
// shape; the first launch of a shape on an uncaptured stream times each of
// them (HIP events, kSearchReps launches into the caller's own D) and keeps
// the fastest (VOSDET_GEMM_SEARCH=0: the heuristic's first choice).  The
// memory-bound bottleneck shapes (K = 64..256 with the residual) are where the
// first choice is worst (tools/conv_roofline.py, profiles/r02_conv_roofline*).
// For those shapes the search also times the hand-written MFMA kernel
// (gemm1x1.hip) and keeps it when it is faster; VOSDET_GEMM_MFMA=1 forces it
// (where supported), =0 excludes it.
//
// Pinned choices (the timed search may pick different kernels --
// different summation orders -- in different processes): VOSDET_GEMM_PLANS
// names a text file of "M N K relu has_res choice" lines (choice = "own" or
// "blas <i>", i = the index in hipBLASLt's heuristic list for the shape, stable
// for one library build and GPU).  A listed shape uses its choice without a
// search, so every process that reads the same file -- the GPU tests and the
// bench, every rank of a multi-GPU run -- computes the same numbers.  With
// VOSDET_GEMM_PLANS_RECORD=1 the result of each new search is appended to it.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <stdlib.h>

#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <tuple>

#include "vosdet_internal.hpp"

namespace vd {

namespace {

constexpr int kMaxAlgos = 64, kSearchReps = 3;
// candidates asked of the heuristic (VOSDET_GEMM_MAXALGOS, default 16, <= kMaxAlgos):
// pinned indices name entries of this list
int max_algos() {
    static int n = 0;
    if (!n) {
        const char *e = getenv("VOSDET_GEMM_MAXALGOS");
        n = e ? atoi(e) : 16;
        if (n < 1) n = 1;
        if (n > kMaxAlgos) n = kMaxAlgos;
    }
    return n;
}

struct Plan {
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
    hipblasLtMatmulHeuristicResult_t cand[kMaxAlgos];
    int ncand = 0;
    hipblasLtMatmulAlgo_t algo;
    size_t ws = 0;
    bool ok = false, searched = false;
    bool own = false;  // the hand-written MFMA kernel won the search
};

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
typedef std::tuple<int, int, int, int, int> Key;  // (M, N, K, relu, has_res)
std::map<Key, Plan> g_plans;
std::map<Key, int> g_pinned;  // -1: the MFMA kernel, i >= 0: heuristic candidate i
bool g_pins_loaded = false;

hipblasLtHandle_t handle();

// The plans' validity key: a pinned index names an entry of hipBLASLt's heuristic
// list, which is stable only for one library build on one GPU.  The
// file carries "# key <arch> hipblaslt-<version>-<git revision> cu<CUs>" lines; a pin
// applies only under a key line equal to this process's key, so on another GPU or
// hipBLASLt build every shape falls back to the timing search instead of silently
// running whatever kernel the stale index now names.
const char *plans_key() {
    static char key[256] = {0};
    if (key[0]) return key;
    hipDeviceProp_t prop;
    int dev = 0, ver = 0;
    char rev[128] = {0};
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return "";
    if (hipblasLtHandle_t h = handle()) {
        (void)hipblasLtGetVersion(h, &ver);
        (void)hipblasLtGetGitRevision(h, rev);
    }
    char arch[64];
    snprintf(arch, sizeof arch, "%s", prop.gcnArchName);
    if (char *c = strchr(arch, ':')) *c = 0;  // gfx950[:sramecc+:xnack-] -> gfx950
    for (char *c = rev; *c; ++c)
        if (*c == ' ' || *c == '\n') *c = '_';
    snprintf(key, sizeof key, "%s hipblaslt-%d-%s cu%d", arch, ver, rev[0] ? rev : "0",
             prop.multiProcessorCount);
    return key;
}

bool g_key_in_file = false;  // the file already has this process's key line

void load_pins() {  // once, under g_mu
    if (g_pins_loaded) return;
    g_pins_loaded = true;
    const char *path = getenv("VOSDET_GEMM_PLANS");
    if (!path || !path[0]) return;
    FILE *f = fopen(path, "r");
    if (!f) return;
    const char *mine = plans_key();
    bool active = false;  // pins before any key line (or under another key) never apply
    char line[512];
    while (fgets(line, sizeof line, f)) {
        if (strncmp(line, "# key ", 6) == 0) {
            char *e = line + strlen(line);
            while (e > line && (e[-1] == '\n' || e[-1] == '\r' || e[-1] == ' ')) *--e = 0;
            active = mine[0] && strcmp(line + 6, mine) == 0;
            g_key_in_file |= active;
            continue;
        }
        if (!active || line[0] == '#') continue;
        int M, N, K, relu, res, idx = 0;
        char what[16];
        const int n = sscanf(line, "%d %d %d %d %d %15s %d", &M, &N, &K, &relu, &res, what, &idx);
        if (n >= 6 && strcmp(what, "own") == 0)
            g_pinned[Key(M, N, K, relu, res)] = -1;
        else if (n == 7 && strcmp(what, "blas") == 0 && idx >= 0)
            g_pinned[Key(M, N, K, relu, res)] = idx;
    }
    fclose(f);
}

void record_pin(const Key &k, int choice) {
    const char *rec = getenv("VOSDET_GEMM_PLANS_RECORD");
    const char *path = getenv("VOSDET_GEMM_PLANS");
    if (!rec || rec[0] != '1' || !path || !path[0]) return;
    FILE *f = fopen(path, "a");
    if (!f) return;
    if (!g_key_in_file && plans_key()[0]) {  // this process's pins go under its key
        fprintf(f, "# key %s\n", plans_key());
        g_key_in_file = true;
    }
    if (choice < 0)
        fprintf(f, "%d %d %d %d %d own\n", std::get<0>(k), std::get<1>(k), std::get<2>(k),
                std::get<3>(k), std::get<4>(k));
    else
        fprintf(f, "%d %d %d %d %d blas %d\n", std::get<0>(k), std::get<1>(k), std::get<2>(k),
                std::get<3>(k), std::get<4>(k), choice);
    fclose(f);
}

constexpr size_t kMaxWs = 64ull << 20;

hipblasLtHandle_t handle() {
    if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) g_handle = nullptr;
    return g_handle;
}

Plan *plan_for(int M, int N, int K, int relu, int has_res) {
    load_pins();
    auto key = std::make_tuple(M, N, K, relu, has_res);
    auto it = g_plans.find(key);
    if (it != g_plans.end()) return it->second.ok ? &it->second : nullptr;
    Plan &p = g_plans[key];
    hipblasLtHandle_t h = handle();
    if (!h) return nullptr;
    if (hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
        return nullptr;
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtEpilogue_t epi = relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS;
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
    hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    // a dummy bias pointer for the heuristic query (set per call)
    if (hipblasLtMatrixLayoutCreate(&p.a, HIP_R_32F, K, N, K) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.b, HIP_R_32F, K, M, K) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.c, HIP_R_32F, N, M, N) != HIPBLAS_STATUS_SUCCESS)
        return nullptr;
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    uint64_t wsmax = kMaxWs;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax,
                                          sizeof(wsmax));
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.op, p.a, p.b, p.c, p.c, pref,
                                                               max_algos(), p.cand, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return nullptr;
    p.ncand = n;
    p.algo = p.cand[0].algo;
    p.ws = p.cand[0].workspaceSize;
    p.ok = true;
    auto pin = g_pinned.find(key);
    if (pin != g_pinned.end()) {  // a pinned choice: no timing search
        if (pin->second < 0 && gemm1x1_mfma_supported(K, N)) {
            p.own = true;
            p.searched = true;
        } else if (pin->second >= 0 && pin->second < n) {
            p.algo = p.cand[pin->second].algo;
            p.ws = p.cand[pin->second].workspaceSize;
            p.searched = true;
        }
    }
    return &p;
}

bool search_enabled() {
    const char *e = getenv("VOSDET_GEMM_SEARCH");
    return !(e && e[0] == '0');
}

int own_mode() {  // -1: never, 0: when it wins the search, 1: always (where supported)
    const char *e = getenv("VOSDET_GEMM_MFMA");
    return !e ? 0 : (e[0] == '0' ? -1 : 1);
}

// Time every candidate on the caller's operands (D is overwritten by the real
// launch that follows) and keep the fastest; any failure keeps the heuristic's
// first choice.
void search(Plan &p, int M, int N, int K, int relu, const float *A, const float *W,
            const float *bias, const float *R, float *D, void *ws, size_t ws_bytes, hipStream_t s) {
    p.searched = true;
    const bool try_own = own_mode() == 0 && gemm1x1_mfma_supported(K, N);
    if ((p.ncand < 2 && !try_own) || !search_enabled()) return;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return;
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return;
    }
    const float alpha = 1.f, beta = R ? 1.f : 0.f;
    float best = 1e30f;
    int best_i = -1;
    for (int i = 0; i < p.ncand; ++i) {
        const hipblasLtMatmulHeuristicResult_t &c = p.cand[i];
        if (c.state != HIPBLAS_STATUS_SUCCESS || c.workspaceSize > ws_bytes ||
            (c.workspaceSize && !ws))
            continue;
        auto launch = [&]() {
            return hipblasLtMatmul(handle(), p.op, &alpha, W, p.a, A, p.b, &beta, R ? R : D, p.c,
                                   D, p.c, &c.algo, ws, c.workspaceSize, s);
        };
        if (launch() != HIPBLAS_STATUS_SUCCESS) continue;  // warm-up / validity
        bool ok = hipEventRecord(e0, s) == hipSuccess;
        for (int r = 0; ok && r < kSearchReps; ++r) ok = launch() == HIPBLAS_STATUS_SUCCESS;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess;
        float ms = 0.f;
        if (ok && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < best) {
            best = ms;
            best_i = i;
        }
    }
    if (try_own && launch_gemm1x1_mfma(A, M, K, W, N, bias, R, relu, D, s) == VD_OK) {
        bool ok = hipEventRecord(e0, s) == hipSuccess;
        for (int r = 0; ok && r < kSearchReps; ++r)
            ok = launch_gemm1x1_mfma(A, M, K, W, N, bias, R, relu, D, s) == VD_OK;
        ok = ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess;
        float ms = 0.f;
        if (ok && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < best) {
            best = ms;
            p.own = true;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipGetLastError();
    if (best_i >= 0 && !p.own) {
        p.algo = p.cand[best_i].algo;
        p.ws = p.cand[best_i].workspaceSize;
    }
    record_pin(Key(M, N, K, relu, R ? 1 : 0), p.own ? -1 : (best_i >= 0 ? best_i : 0));
}

}  // namespace

size_t gemm_epi_workspace_bytes() { return kMaxWs; }

int gemm_plans_key(char *buf, int n) {
    std::lock_guard<std::mutex> g(g_mu);
    const char *k = plans_key();
    if (!k[0]) return VD_ERR_LAUNCH;
    snprintf(buf, (size_t)n, "%s", k);
    return VD_OK;
}

// One line per planned shape: "M N K relu has_res own|blas ws_bytes".  A
// hipBLASLt algorithm with ws_bytes > 0 keeps split-K partials / stream-K
// fix-up state in the caller's workspace between its workgroups, so two GEMMs
// given the same workspace must never run at the same time.
int gemm_plan_list(char *buf, int n) {
    std::lock_guard<std::mutex> g(g_mu);
    if (!buf || n < 1) return VD_ERR_ARG;
    int used = 0;
    buf[0] = 0;
    for (const auto &kv : g_plans) {
        const Plan &p = kv.second;
        if (!p.ok) continue;
        const int w = snprintf(buf + used, (size_t)(n - used), "%d %d %d %d %d %s %zu\n",
                               std::get<0>(kv.first), std::get<1>(kv.first),
                               std::get<2>(kv.first), std::get<3>(kv.first),
                               std::get<4>(kv.first), p.own ? "own" : "blas",
                               p.own ? (size_t)0 : p.ws);
        if (w < 0 || w >= n - used) return VD_ERR_WORKSPACE;  // buffer too small
        used += w;
    }
    return VD_OK;
}

int launch_gemm_bias_act(const float *A, int M, int K, const float *W, int N, const float *bias,
                         const float *R, int relu, float *D, void *ws, size_t ws_bytes,
                         hipStream_t s) {
    if (M == 0) return VD_OK;
    const int mode = own_mode();
    if (mode == 1 && gemm1x1_mfma_supported(K, N))
        return launch_gemm1x1_mfma(A, M, K, W, N, bias, R, relu, D, s);
    std::lock_guard<std::mutex> lk(g_mu);
    Plan *p = plan_for(M, N, K, relu ? 1 : 0, R ? 1 : 0);
    if (!p) return VD_ERR_SHAPE;
    hipblasLtMatmulDescSetAttribute(p->op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                    sizeof(bias));
    if (!p->searched) search(*p, M, N, K, relu ? 1 : 0, A, W, bias, R, D, ws, ws_bytes, s);
    if (p->own && mode == 0) return launch_gemm1x1_mfma(A, M, K, W, N, bias, R, relu, D, s);
    if (p->ws > ws_bytes || (p->ws && !ws)) return VD_ERR_WORKSPACE;
    const float alpha = 1.f, beta = R ? 1.f : 0.f;
    const hipblasStatus_t st =
        hipblasLtMatmul(handle(), p->op, &alpha, W, p->a, A, p->b, &beta, R ? R : D, p->c, D,
                        p->c, &p->algo, ws, p->ws, s);
    return st == HIPBLAS_STATUS_SUCCESS ? VD_OK : VD_ERR_LAUNCH;
}

}  // namespace vd
