// trace_planner.hip -- anatomy of the block planner's steps (k_blk_step<L>, csrc/smx_block.hpp):
// the library built with SMX_BLK_TRACE (per-workgroup s_memrealtime stamps at 8 phases of every
// step), one block of P pivots planned on a seeded N x N table (uniform LP: A ~ U(-1, 1),
// b ~ U(0.1, 1), f ~ U(-1, 1), so every step is a phase-2 ratio test), printed as one JSON line
// per step: median over the workgroups of each phase's end relative to the step's earliest
// entry stamp (us), and the step's span.
//
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSMX_BLK_TRACE -Iinclude \
//     -I/opt/rocm/include -L/opt/rocm/lib -lrccl tools/trace_planner.hip -o tools/trace_planner
// Run: tools/trace_planner [N] [P] [blocks] [planner: 0 window (persistent where eligible,
//   the default), 2 window launch form, 1 register] [nwin]
#include "../simplex-method-solver_amd/csrc/smx_kernels.hip"

#include <algorithm>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

namespace {
__global__ void k_lp(double* T, int64_t ld, int n, int m, unsigned long long seed) {
    const int64_t total = (int64_t)(n + 1) * ld;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / ld, j = t % ld;
        unsigned long long z = (uint64_t)t * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const double u = (double)(z >> 11) * 0x1p-53;
        double v = 0.0;
        if (j < m) v = 2.0 * u - 1.0;
        else if (j == m && i < n) v = 0.1 + 0.9 * u;
        T[t] = v;
    }
}
}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int P = argc > 2 ? atoi(argv[2]) : 12;
    const int nblocks = argc > 3 ? atoi(argv[3]) : 3;
    if (argc > 4) smx_tune_block_planner(atoi(argv[4]), argc > 5 ? atoi(argv[5]) : 0);
    smx_shape s{};
    s.m = N - 1;
    s.n = s.rows = N - 1;
    s.flen = s.m;
    s.row0 = 0;
    s.ld = (N + 15) / 16 * 16;
    s.nparts = smx_nparts_for(s.rows, s.m);
    const size_t nb = (size_t)N * s.ld * 8;
    double *b0, *b1;
    CK(hipMalloc(&b0, nb));
    CK(hipMalloc(&b1, nb));
    smx_ctl* ctl;
    CK(hipMalloc(&ctl, sizeof(smx_ctl)));
    CK(hipMemset(ctl, 0, sizeof(smx_ctl)));
    int32_t pv = P;
    const int64_t bb = smx_block_bytes(&s, &pv);
    void* blk;
    CK(hipMalloc(&blk, bb));
    int32_t* log;
    double* xh;
    CK(hipMalloc(&log, 1 << 20));
    CK(hipMalloc(&xh, 1 << 21));
    hipLaunchKernelGGL(k_lp, dim3(4096), dim3(256), 0, 0, b0, s.ld, s.n, s.m, 7ull);
    CK(hipDeviceSynchronize());
    CK((hipError_t)smx_reset(b0, &s, 0, 1, ctl, nullptr));
    int parity = 0;
    for (int rep = 0; rep < nblocks; ++rep) {
        CK((hipError_t)smx_block_run(b0, b1, &s, parity, P, P, ctl, blk, bb, log, xh, 1 << 17,
                                     nullptr));
        CK(hipDeviceSynchronize());
        parity = (parity + P) & 1;
        static unsigned long long tr[kBlkMax + 1][kBlkTraceParts][kBlkTracePh];
        CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_blk_trace), sizeof(tr)));
        {
            static const unsigned long long z[kBlkMax + 1][kBlkTraceParts][kBlkTracePh] = {};
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_blk_trace), z, sizeof(z)));
        }
        static unsigned fb[kBlkMax + 1][2];
        CK(hipMemcpyFromSymbol(fb, HIP_SYMBOL(g_blk_fallback), sizeof(fb)));
        {
            static const unsigned zero[kBlkMax + 1][2] = {};
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_blk_fallback), zero, sizeof(zero)));
        }
        // the first kBlkTraceParts planner workgroups (window planner: phases 0 entry, 1 decision,
        // 2 pivot element, 3 next entering column, 4 bookkeeping, 5 row pass, 7 records stored)
        const int Gp = g_block_planner != 1 ? win_groups(s.rows) : blk_parts_of(s.nparts, s.rows);
        const int G = Gp < kBlkTraceParts ? Gp : kBlkTraceParts;
        unsigned long long prev_end = 0;
        for (int L = 1; L <= P; ++L) {
            unsigned long long t0 = ~0ull, tend = 0;
            for (int g = 0; g < G; ++g) {
                t0 = std::min(t0, tr[L][g][0]);
                tend = std::max(tend, tr[L][g][7]);
            }
            // gap: this step's first entry after the previous step's last record store
            const double gap = prev_end ? ((double)t0 - (double)prev_end) * 0.01 : 0.0;
            prev_end = tend;
            printf("{\"rep\": %d, \"N\": %d, \"P\": %d, \"L\": %d, \"span_us\": %.2f, "
                   "\"gap_us\": %.2f, \"phase_us\": [",
                   rep, N, P, L, (tend - t0) * 0.01, gap);
            for (int ph = 0; ph < kBlkTracePh; ++ph) {
                std::vector<double> v;
                for (int g = 0; g < G; ++g)
                    if (tr[L][g][ph]) v.push_back((tr[L][g][ph] - t0) * 0.01);
                if (v.empty()) v.push_back(-1.0);
                std::sort(v.begin(), v.end());
                printf("%s%.2f", ph ? ", " : "", v[v.size() / 2]);
            }
            printf("], \"fallback_waves\": [%u, %u]}\n", fb[L][0], fb[L][1]);
        }
    }
    return 0;
}
