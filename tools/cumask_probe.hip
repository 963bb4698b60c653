// cumask_probe.hip -- can the block planner get CUs of its own?  (pipelined chains)
// Streams created with hipExtStreamCreateWithCUMask: which CUs (XCC_ID, HW_ID) a masked stream's
// workgroups land on, how a fp64-issue-bound kernel (the sweep's stand-in) scales with the CUs it
// is given, and how a latency-bound kernel of 64 workgroups (the planner's stand-in: dependent
// global loads) runs alone and beside the issue-bound one, masked and unmasked.
// Mask: r CUs per XCD for the planner, bits {32x + x + 8t : x < 8, t < r} -- r per XCD whether the
// driver maps bit i to XCD i / 32 or to XCD i % 8.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/cumask_probe tools/cumask_probe.hip
//   run:   tools/cumask_probe   (JSON lines)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <set>
#include <map>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,              \
                    hipGetErrorString(e_));                                        \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ void k_who(unsigned* out, unsigned spin_ticks) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

// fp64 issue: 8 independent FMA chains per lane
__global__ void k_valu(double* out, int iters) {
    double a[8];
    for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-9 + k;
    const double m = 0.999999, c = 1e-7;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fma(a[k], m, c);
    double s = 0;
    for (int k = 0; k < 8; ++k) s += a[k];
    if (s == 12345.678) out[blockIdx.x] = s;   // never: keeps the chains alive
}

// dependent loads: each lane chases its own index chain through a large buffer
__global__ void k_chase(const int* __restrict__ nxt, int* out, int steps) {
    int i = (blockIdx.x * blockDim.x + threadIdx.x) * 97;
    for (int s = 0; s < steps; ++s) i = nxt[i];
    if (i == -7) out[0] = i;
}

static std::vector<uint32_t> plan_mask(int ncu, int r, bool complement) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0);
    std::set<int> s;
    for (int x = 0; x < 8; ++x)
        for (int t = 0; t < r; ++t) s.insert(32 * x + x + 8 * t);
    for (int i = 0; i < ncu; ++i) {
        const bool in = s.count(i) > 0;
        if (in != complement) m[i / 32] |= 1u << (i % 32);
    }
    return m;
}

static hipStream_t mk(int ncu, int r, bool complement) {
    hipStream_t s;
    if (r < 0) {
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return s;
    }
    std::vector<uint32_t> m = plan_mask(ncu, r, complement);
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    return s;
}

static void who(hipStream_t s, const char* name, int r, int nwg) {
    unsigned* d;
    CK(hipMalloc(&d, sizeof(unsigned) * 2 * nwg));
    hipLaunchKernelGGL(k_who, dim3(nwg), dim3(64), 0, s, d, 2000u);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned> h(2 * nwg);
    CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
    std::set<std::pair<unsigned, unsigned>> cus;
    std::map<unsigned, std::set<unsigned>> per;
    for (int b = 0; b < nwg; ++b) {
        const unsigned xcc = h[2 * b] & 0xf, hw = h[2 * b + 1];
        const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        const unsigned id = (se << 5) | (sh << 4) | cu;
        cus.insert({xcc, id});
        per[xcc].insert(id);
    }
    printf("{\"probe\": \"who\", \"stream\": \"%s\", \"r\": %d, \"wgs\": %d, \"distinct_cus\": %zu, \"per_xcc\": {",
           name, r, nwg, cus.size());
    bool first = true;
    for (auto& kv : per) {
        printf("%s\"%u\": %zu", first ? "" : ", ", kv.first, kv.second.size());
        first = false;
    }
    printf("}}\n");
    CK(hipFree(d));
}

static float time_on(hipStream_t s, void (*launch)(hipStream_t)) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    launch(s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms;
}

static double* g_out;
static int* g_nxt;
static int* g_iout;
static int g_valu_wgs = 2048, g_valu_iters = 20000, g_chase_steps = 400;
static void launch_valu(hipStream_t s) {
    hipLaunchKernelGGL(k_valu, dim3(g_valu_wgs), dim3(256), 0, s, g_out, g_valu_iters);
}
static void launch_chase(hipStream_t s) {
    hipLaunchKernelGGL(k_chase, dim3(64), dim3(256), 0, s, (const int*)g_nxt, g_iout, g_chase_steps);
}

// both kernels at once on two streams; times of each (events on its own stream)
static void pair(hipStream_t sv, hipStream_t sc, const char* name, int r) {
    hipEvent_t a0, a1, b0, b1;
    CK(hipEventCreate(&a0));
    CK(hipEventCreate(&a1));
    CK(hipEventCreate(&b0));
    CK(hipEventCreate(&b1));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a0, sv));
    launch_valu(sv);
    CK(hipEventRecord(a1, sv));
    // the latency kernel starts once the issue-bound one has filled its CUs
    CK(hipEventRecord(b0, sc));
    launch_chase(sc);
    CK(hipEventRecord(b1, sc));
    CK(hipDeviceSynchronize());
    float tv = 0, tc = 0, tcs = 0;
    CK(hipEventElapsedTime(&tv, a0, a1));
    CK(hipEventElapsedTime(&tc, b0, b1));
    CK(hipEventElapsedTime(&tcs, a0, b0));
    printf("{\"probe\": \"pair\", \"streams\": \"%s\", \"r\": %d, \"valu_ms\": %.4f, \"chase_ms\": %.4f, \"chase_start_ms\": %.4f}\n",
           name, r, tv, tc, tcs);
    CK(hipEventDestroy(a0));
    CK(hipEventDestroy(a1));
    CK(hipEventDestroy(b0));
    CK(hipEventDestroy(b1));
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"probe\": \"device\", \"cus\": %d}\n", ncu);
    CK(hipMalloc(&g_out, sizeof(double) * 65536));
    const size_t N = 16u << 20;   // 64 MiB of indices
    std::vector<int> h(N);
    uint64_t x = 88172645463325252ull;
    for (size_t i = 0; i < N; ++i) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        h[i] = (int)(x % N);
    }
    CK(hipMalloc(&g_nxt, N * sizeof(int)));
    CK(hipMalloc(&g_iout, 64));
    CK(hipMemcpy(g_nxt, h.data(), N * sizeof(int), hipMemcpyHostToDevice));

    hipStream_t full = mk(ncu, -1, false);
    who(full, "unmasked", 0, 4096);
    for (int r : {1, 2, 4}) {
        hipStream_t p = mk(ncu, r, false), sw = mk(ncu, r, true);
        who(p, "planner", r, 1024);
        who(sw, "sweep", r, 4096);
        CK(hipStreamDestroy(p));
        CK(hipStreamDestroy(sw));
    }
    // warm
    (void)time_on(full, launch_valu);
    (void)time_on(full, launch_chase);
    printf("{\"probe\": \"alone\", \"stream\": \"unmasked\", \"valu_ms\": %.4f, \"chase_ms\": %.4f}\n",
           time_on(full, launch_valu), time_on(full, launch_chase));
    for (int r : {1, 2, 4}) {
        hipStream_t p = mk(ncu, r, false), sw = mk(ncu, r, true);
        const int keep = g_valu_wgs;
        g_valu_wgs = 8 * (ncu - 8 * r);   // the sweep's grid sized for its CUs
        printf("{\"probe\": \"alone\", \"stream\": \"masked\", \"r\": %d, \"valu_wgs\": %d, \"valu_ms\": %.4f, \"chase_ms\": %.4f}\n",
               r, g_valu_wgs, time_on(sw, launch_valu), time_on(p, launch_chase));
        pair(sw, p, "masked", r);
        g_valu_wgs = keep;
        CK(hipStreamDestroy(p));
        CK(hipStreamDestroy(sw));
    }
    hipStream_t other = mk(ncu, -1, false);
    pair(full, other, "unmasked", 0);
    CK(hipStreamDestroy(other));
    CK(hipStreamDestroy(full));
    return 0;
}
