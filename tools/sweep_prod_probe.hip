// sweep_prod_probe.hip -- the production flag-form sweep (k_blk_sweep<P, true, 4>, csrc/smx_block.hpp)
// timed on the synthetic operands of tools/sweep_lab.hip, to separate code from data effects.
//   mode 0: no pivot rows, no pivot columns inside the table (h->r = -1, h->c = C + q)
//   mode 1: pivot rows / columns as a real block would have them (rows (q*977+5) % R, columns
//           (q*1231+7) % C), flags from the multipliers; k_blk_sweep_rest (blk_fixcols) after it
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -I/opt/rocm/include \
//     -L/opt/rocm/lib -lrccl tools/sweep_prod_probe.hip -o tools/sweep_prod_probe
// Run: tools/sweep_prod_probe [N=16384] [reps=5] [bpc=7]
#include "../simplex-method-solver_amd/csrc/smx_kernels.hip"

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

namespace {

__global__ void k_fill(double* p, int64_t n, unsigned long long seed, double lo, double hi) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed * 0xD1B54A32D192ED03ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = lo + (hi - lo) * (double)(z >> 11) * 0x1p-53;
    }
}

__global__ void k_hdr(BlkHdr* h, int P, int R, int C, int mode) {
    if (threadIdx.x != 0) return;
    h->peff = P;
    h->loc = 0;
    for (int q = 0; q < kBlkMax; ++q) {
        h->r[q] = mode ? (q * 977 + 5) % (R - 1) : -1;
        h->c[q] = mode ? (q * 1231 + 7) % C : C + q;
        const double e = (q & 1 ? -1.0 : 1.0) * (0.6 + 0.1 * q);
        const FastDiv fd = fd_prep(e);
        h->e[q] = e;
        h->y[q] = fd.y;
        h->ok[q] = fd.ok ? 1 : 0;
    }
}

__global__ void k_flags(const double* mul, const BlkHdr* h, int R, int P, int32_t* f) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R; i += gridDim.x * blockDim.x) {
        uint32_t mt = 0;
        bool piv = false;
        for (int q = 0; q < P; ++q) {
            mt = max(mt, bnd_term(mul[(int64_t)i * kBlkMax + q]));
            piv = piv || i == h->r[q];
        }
        f[i] = (mt < kBndSpan && !piv) ? 1 : 0;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int bpc = argc > 3 ? atoi(argv[3]) : 7;
    const int R = N, C = N;
    const int64_t ld = C;
    const int64_t nel = (int64_t)R * ld;
    smx_shape s{};
    s.ld = ld;
    s.rows = R - 1;
    s.n = R - 1;
    s.m = C - 1;
    s.flen = C - 1;
    s.row0 = 0;
    s.nparts = 64;
    const BlkLayout L = blk_layout(R, ld, 64);
    double *T0, *T, *other;
    char* blk;
    CK(hipMalloc(&T0, nel * 8));
    CK(hipMalloc(&T, nel * 8));
    CK(hipMalloc(&other, 64));
    CK(hipMalloc(&blk, L.bytes));
    CK(hipMemset(blk, 0, L.bytes));
    BlkHdr* h = reinterpret_cast<BlkHdr*>(blk);
    double* mul = reinterpret_cast<double*>(blk + L.mul);
    double* pr = reinterpret_cast<double*>(blk + L.pr);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, T0, nel, 1ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, pr, (int64_t)kBlkMax * ld, 2ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, mul, (int64_t)R * kBlkMax, 3ull, -1.0, 1.0);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int P : {10, 12}) {
        for (int mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(k_hdr, dim3(1), dim3(64), 0, 0, h, P, R, C, mode);
            hipLaunchKernelGGL(k_flags, dim3(64), dim3(256), 0, 0, mul, h, R, P,
                               blk_rflags(mul, R));
            CK(hipDeviceSynchronize());
            std::vector<float> ms, ms_all;
            for (int r = 0; r < reps + 1; ++r) {
                CK(hipMemcpy(T, T0, nel * 8, hipMemcpyDeviceToDevice));
                CK(hipDeviceSynchronize());
                BlkSweepFn fn = blk_sweep_fn(P, true, 4);
                const int grid = num_cus() * bpc - (num_cus() * bpc) % 128;
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(fn, dim3(grid), dim3(kUpdBlock), 0, 0, T, other, ld, R, C,
                                   (const BlkHdr*)h, (const double*)mul, (const double*)pr, h, 0,
                                   0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (r > 0) ms.push_back(t);
                if (mode == 0) continue;   // blk_fixcols needs pivot columns inside the table
                CK(hipEventRecord(e0, 0));
                launch_block_sweep(T, other, s, P, blk, L, 0, 0, 0, 0, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&t, e0, e1));
                if (r > 0) ms_all.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            std::sort(ms_all.begin(), ms_all.end());
            printf("{\"N\": %d, \"P\": %d, \"mode\": %d, \"bpc\": %d, \"sweep_best_us\": %.1f, "
                   "\"sweep_median_us\": %.1f, \"launch_block_sweep_best_us\": %.1f}\n",
                   N, P, mode, bpc, ms[0] * 1e3, ms[ms.size() / 2] * 1e3,
                   ms_all.empty() ? 0.0 : ms_all[0] * 1e3);
            fflush(stdout);
        }
    }
    return 0;
}
