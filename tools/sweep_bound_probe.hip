// sweep_bound_probe.hip -- what bounds the one-row-per-batch block sweep (blk_sweep_body_row1,
// csrc/smx_block.hpp) at P = 10 / 12, and whether LDS-DMA staging lifts it.
//
// Variants (template MODE of k_bnd; the row body is the production one, restated here so the
// load path can change):
//   0 prod    the production loop (next row's load issued before this row's arithmetic)
//   1 noload  arithmetic and stores only: the row's values come from registers (no HBM reads;
//             results differ, not compared)
//   2 copy    loads and stores only (no arithmetic; not compared)
//   3 mulpf   as 0, with the next row's multipliers loaded before this row's arithmetic
//   4 glds    rows staged global -> LDS by global_load_lds_dwordx4 (no VGPR destination), D rows
//             ahead per wave in an LDS ring; ds_read_b128 of the row before its arithmetic
//   5 nostore loads and arithmetic, no stores (not compared)
//   6 plainstore  as 0 with temporal stores;  7 tload  as 0 with temporal loads
// (modes 3 and 4 were measured in the first run, profiles/r02/sweep_bound_probe_P*.jsonl)
// Every compared variant is checked bit for bit against the production sweep's output.
//
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -I/opt/rocm/include \
//     -L/opt/rocm/lib -lrccl tools/sweep_bound_probe.hip -o tools/sweep_bound_probe
// Run: tools/sweep_bound_probe [N=16384] [P=12]
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

__global__ void k_hdr(BlkHdr* h, int P, int R, int C) {
    if (threadIdx.x != 0) return;
    h->peff = P;
    for (int q = 0; q < kBlkMax; ++q) {
        h->r[q] = (q * 977 + 5) % (R - 1);
        h->c[q] = (q * 1231 + 7) % C;
        const double e = (q & 1 ? -1.0 : 1.0) * (0.6 + 0.1 * q);
        const FastDiv fd = fd_prep(e);
        h->e[q] = e;
        h->y[q] = fd.y;
        h->ok[q] = fd.ok ? 1 : 0;
    }
}

__global__ void k_cmp(const double* a, const double* b, int64_t ld, int R, int C,
                      unsigned long long* bad) {
    unsigned long long n = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < (int64_t)R * C;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / C, j = t % C;
        n += __double_as_longlong(a[i * ld + j]) != __double_as_longlong(b[i * ld + j]);
    }
    if (n) atomicAdd(bad, n);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt before row k's ring slot is read: D-1+k for the first D rows (prologue loads, then a
// load and a store per row consumed), 2D-1 in the steady state (the store of row k-D, then a
// load and a store for each of the D-1 rows between)
template <int D, int K = 0>
__device__ __forceinline__ void wait_slot(int k) {
    if constexpr (K == D) {
        wait_vm<2 * D - 1>();
    } else {
        if (k == K)
            wait_vm<D - 1 + K>();
        else
            wait_slot<D, K + 1>(k);
    }
}

template <int P, int MODE, int D>
__global__ __launch_bounds__(kUpdBlock) void k_bnd(double* Tin, double* Tout, int64_t ld, int R,
                                                   int C, const BlkHdr* __restrict__ h,
                                                   const double* __restrict__ mul,
                                                   const double* __restrict__ pr) {
    __shared__ dbl2 ring[MODE == 4 ? kUpdWaves : 1][MODE == 4 ? D : 1][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int rq[P], cq[P];
    double eq[P], yq[P];
    bool allok = true;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        rq[q] = h->r[q];
        cq[q] = h->c[q];
        eq[q] = h->e[q];
        yq[q] = h->y[q];
        allok = allok && h->ok[q] != 0;
    }
    constexpr int kChunk = 2 * kWave;
    const int NW = (int)gridDim.x * kUpdWaves;
    const int w = (int)blockIdx.x * kUpdWaves + wv;
    const int nchunks = (C + kChunk - 1) / kChunk;
    const int qs = NW / nchunks;
    const int ch = w % nchunks;
    const int j = ch * kChunk + 2 * lane;
    const int c0 = ch * kChunk;
    dbl2 prs[P];
    bool colchunk = false;
    uint32_t cbits = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        prs[q] = (j < C) ? *reinterpret_cast<const dbl2*>(pr + (int64_t)q * ld + j)
                         : dbl2{0.0, 0.0};
        colchunk = colchunk || (cq[q] >= c0 && cq[q] < c0 + kChunk);
        cbits |= (cq[q] == j ? 1u : 0u) << (2 * q);
        cbits |= (cq[q] == j + 1 ? 1u : 0u) << (2 * q + 1);
    }
    const bool cspecial = !allok;
    const int base = w / nchunks;
    const int tbq = blk_special_batch<P, 1>(h, base, qs);
    int tsp = blk_next_batch<P>(tbq, -1);
    double pcn[P];
    auto row1 = [&](dbl2 x0, int i0, int t) {
        const double* m0 = mul + (int64_t)i0 * kBlkMax;
        double pc0[P];
        const bool special = cspecial || t == tsp;
        if (t == tsp) tsp = blk_next_batch<P>(tbq, t);
        if constexpr (MODE == 3) {
#pragma unroll
            for (int q = 0; q < P; ++q) pc0[q] = pcn[q];
            const double* mn = mul + (int64_t)min(i0 + qs, R - 1) * kBlkMax;
#pragma unroll
            for (int q = 0; q < P; ++q) pcn[q] = mn[q];
        } else {
#pragma unroll
            for (int q = 0; q < P; ++q) pc0[q] = m0[q];
        }
        dbl2 v0 = x0;
        bool ok = false;
        auto fast = [&](auto selc) {
            constexpr bool SEL = decltype(selc)::value;
            uint32_t wt = 0;
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const double e = eq[q], y = yq[q];
                double n[2];
                n[0] = v0[0] * e - prs[q][0] * pc0[q];
                n[1] = v0[1] * e - prs[q][1] * pc0[q];
                if (SEL) {
                    const bool s0 = (cbits >> (2 * q)) & 1u, s1 = (cbits >> (2 * q + 1)) & 1u;
                    n[0] = s0 ? v0[0] : n[0];
                    n[1] = s1 ? v0[1] : n[1];
                }
                double rr[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    wt = max(wt, win_term(n[k]));
                    const double tq = n[k] * y;
                    const double r = fma(-e, tq, n[k]);
                    rr[k] = fma(r, y, tq);
                }
                v0 = dbl2{rr[0], rr[1]};
            }
            ok = __all(wt < kWinSpan);
        };
        if constexpr (MODE == 2) {
            ok = true;
        } else {
            if (!special) {
                if (colchunk)
                    fast(SmxBool<true>{});
                else
                    fast(SmxBool<false>{});
            }
        }
        if (!ok) {
            const int jl = min(j, (C - 1) & ~1);
            x0 = *reinterpret_cast<const dbl2*>(Tin + (int64_t)i0 * ld + jl);
            v0 = blk_exact<P>(x0, i0, j, rq, cq, eq, prs, pc0);
        }
        if constexpr (MODE == 5) {
            // loads and arithmetic, no stores: the store is kept only for a value the table never
            // holds (so the arithmetic is not dead code)
            if (j < C && v0[0] == 1234567.0)
                __builtin_nontemporal_store(v0, reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j));
        } else if constexpr (MODE == 6) {
            if (j < C) *reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j) = v0;   // plain store
        } else {
            if (j < C)
                __builtin_nontemporal_store(v0, reinterpret_cast<dbl2*>(Tout + (int64_t)i0 * ld + j));
        }
    };
    const int jc = min(j, (C - 1) & ~1);
    if constexpr (MODE == 3) {
        const double* m0 = mul + (int64_t)min(base, R - 1) * kBlkMax;
#pragma unroll
        for (int q = 0; q < P; ++q) pcn[q] = m0[q];
    }
    if constexpr (MODE == 4) {
        // LDS ring: slot s of this wave holds one row's 128 columns, lane-linear (1 KiB)
        auto glds = [&](int row, int slot) {
            const double* p = Tin + (int64_t)min(row, R - 1) * ld + jc;
            const uint32_t dst = __builtin_amdgcn_readfirstlane(
                (uint32_t)(uintptr_t)&ring[wv][slot][0]);
            uint32_t keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(p), "s"(dst)
                         : "memory");
        };
#pragma unroll
        for (int k = 0; k < D; ++k) glds(base + k * qs, k);
        int t = 0, slot = 0;
        for (int i0 = base; i0 < R; i0 += qs, ++t) {
            wait_slot<D>(t);
            const dbl2 x = ring[wv][slot][lane];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            glds(i0 + D * qs, slot);
            slot = slot + 1 == D ? 0 : slot + 1;
            row1(x, i0, t);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    auto ldc = [&](int row) {
        dbl2 v;
        if constexpr (MODE == 1) {
            // values from registers: same magnitude as the table's, inside the window
            v = dbl2{0.25 + 1e-7 * row, -0.5 + 1e-7 * (row + lane)};
        } else {
            const double* p = Tin + (int64_t)min(row, R - 1) * ld + jc;
            if constexpr (MODE == 7)   // temporal loads
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
            else
                asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
        }
        return v;
    };
    dbl2 a = ldc(base), b = ldc(base + qs);
    asm volatile("s_waitcnt vmcnt(1)" : "+v"(a) :: "memory");
    int t = 0;
    for (int i0 = base; i0 < R; i0 += 2 * qs, t += 2) {
        row1(a, i0, t);
        if (i0 + qs >= R) break;
        a = ldc(i0 + 2 * qs);
        asm volatile("s_waitcnt vmcnt(2)" : "+v"(b) :: "memory");
        row1(b, i0 + qs, t + 1);
        if (i0 + 2 * qs >= R) break;
        b = ldc(i0 + 3 * qs);
        asm volatile("s_waitcnt vmcnt(2)" : "+v"(a) :: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

using BndFn = void (*)(double*, double*, int64_t, int, int, const BlkHdr*, const double*,
                       const double*);
struct Var {
    const char* name;
    BndFn fn;
    bool compare;
};

template <int P>
void run(int N) {
    const int R = N, C = N;
    smx_shape s{};
    s.ld = (C + 15) / 16 * 16;
    s.rows = R - 1;
    s.n = R - 1;
    s.m = C - 1;
    s.flen = C - 1;
    s.row0 = 0;
    s.nparts = nparts_for(s.rows, s.m);
    const int64_t ld = s.ld;
    const BlkLayout L = blk_layout(R, ld, s.nparts);
    double *a, *ref, *out;
    char* blk;
    const size_t nb = (size_t)R * ld * 8;
    CK(hipMalloc(&a, nb));
    CK(hipMalloc(&ref, nb));
    CK(hipMalloc(&out, nb));
    CK(hipMalloc(&blk, L.bytes));
    double* mul = reinterpret_cast<double*>(blk + L.mul);
    double* pr = reinterpret_cast<double*>(blk + L.pr);
    BlkHdr* h = reinterpret_cast<BlkHdr*>(blk);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, (int64_t)R * ld, 1ull, -1.0, 1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, pr, (int64_t)kBlkMax * ld, 2ull, -1.0,
                       1.0);
    hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, mul, (int64_t)R * kBlkMax, 3ull, -1.0,
                       1.0);
    hipLaunchKernelGGL(k_hdr, dim3(1), dim3(64), 0, 0, h, P, R, C);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 8;
    auto timeit = [&](auto launch, float* best, float* mean) {
        float b = 1e30f, sum = 0.f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            b = ms < b ? ms : b;
            sum += ms;
        }
        *best = b;
        *mean = sum / reps;
    };
    // production (out of place a -> ref): the reference output and its time
    CK((hipError_t)launch_block_sweep(a, ref, s, P, blk, L, 0, 0, -1));
    CK(hipDeviceSynchronize());
    {
        float best, mean;
        timeit([&] { launch_block_sweep(a, out, s, P, blk, L, 0, 0, -1); }, &best, &mean);
        printf("{\"variant\": \"production\", \"P\": %d, \"best_us\": %.1f, \"mean_us\": %.1f}\n",
               P, best * 1e3, mean * 1e3);
        fflush(stdout);
    }
    unsigned long long* dbad;
    CK(hipMalloc(&dbad, 8));
    const Var vars[] = {
        {"prod", k_bnd<P, 0, 1>, true},     {"noload", k_bnd<P, 1, 1>, false},
        {"copy", k_bnd<P, 2, 1>, false},
        {"nostore", k_bnd<P, 5, 1>, false}, {"plainstore", k_bnd<P, 6, 1>, true},
        {"tload", k_bnd<P, 7, 1>, true},
    };
    const int nchunks = (C + 2 * kWave - 1) / (2 * kWave);
    for (const Var& v : vars) {
        hipFuncAttributes fa;
        CK(hipFuncGetAttributes(&fa, (const void*)v.fn));
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)v.fn, kUpdBlock, 0));
        for (int bpc = occ; bpc <= occ + 2; ++bpc) {
            const int grid = update_grid(s, (const void*)v.fn, 0, bpc);
            if (((int64_t)grid * kUpdWaves) % nchunks != 0) continue;
            auto launch = [&] {
                hipLaunchKernelGGL(v.fn, dim3(grid), dim3(kUpdBlock), 0, 0, a, out, ld, R, C,
                                   (const BlkHdr*)h, (const double*)mul, (const double*)pr);
            };
            unsigned long long bad = 0;
            if (v.compare) {
                CK(hipMemset(out, 0, nb));
                launch();
                CK(hipDeviceSynchronize());
                CK(hipMemset(dbad, 0, 8));
                hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, ref, out, ld, R, C, dbad);
                CK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
            }
            float best, mean;
            timeit(launch, &best, &mean);
            printf("{\"variant\": \"%s\", \"P\": %d, \"bpc\": %d, \"grid\": %d, \"vgpr\": %d, "
                   "\"lds\": %zu, \"occ_api\": %d, \"mismatch\": %llu, \"best_us\": %.1f, "
                   "\"mean_us\": %.1f}\n",
                   v.name, P, bpc, grid, fa.numRegs, fa.sharedSizeBytes, occ, bad, best * 1e3,
                   mean * 1e3);
            fflush(stdout);
        }
    }
    CK(hipFree(dbad));
    CK(hipFree(a));
    CK(hipFree(ref));
    CK(hipFree(out));
    CK(hipFree(blk));
}

}  // namespace

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 16384;
    const int P = argc > 2 ? atoi(argv[2]) : 12;
    if (P == 10)
        run<10>(N);
    else if (P == 8)
        run<8>(N);
    else
        run<12>(N);
    return 0;
}
