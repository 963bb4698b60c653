// Diagnostic: where the time of one fused pivot goes (k_update<kFused>, SMX_TRACE stamps).
// Builds the product kernels from source with -DSMX_TRACE (never the shipped library).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSMX_TRACE -Iinclude \
//         tools/trace_fused.hip -o tools/trace_fused -lrccl
//   tools/trace_fused [size=1024] [pivots=50]
#include "../simplex-method-solver_amd/csrc/smx_kernels.hip"

#include <algorithm>
#include <vector>

static void check(int e, const char* what) {
    if (e) {
        fprintf(stderr, "%s failed: %d\n", what, e);
        exit(1);
    }
}

int main(int argc, char** argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 1024;
    const int K = argc > 2 ? atoi(argv[2]) : 50;
    const int n = S - 1, m = S - 1;
    smx_shape sh{};
    sh.ld = ((m + 1 + 15) / 16) * 16;
    sh.rows = n;
    sh.n = n;
    sh.m = m;
    sh.flen = m;
    sh.row0 = 0;
    sh.nparts = smx_nparts_for(n, m);
    const size_t R = (size_t)n + 1, bytes = R * sh.ld * 8;
    std::vector<double> T(R * sh.ld, 0.0);
    uint64_t x = 88172645463325252ull;   // xorshift: A~U(-1,1), b~U(0.1,1), c~U(-1,1)
    auto u = [&]() {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return (double)(x >> 11) / 9007199254740992.0;
    };
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < m; ++j) T[(size_t)i * sh.ld + j] = 2 * u() - 1;
        T[(size_t)i * sh.ld + m] = 0.1 + 0.9 * u();
    }
    for (int j = 0; j < m; ++j) T[(size_t)n * sh.ld + j] = 2 * u() - 1;
    double *b0, *b1, *xh;
    smx_ctl* ctl;
    smx_part* parts;
    int32_t* log;
    check(hipMalloc(&b0, bytes), "malloc");
    check(hipMalloc(&b1, bytes), "malloc");
    check(hipMalloc(&ctl, sizeof(smx_ctl)), "malloc");
    check(hipMalloc(&parts, 2 * 64 * sizeof(smx_part)), "malloc");
    check(hipMalloc(&log, 2 * 4096 * sizeof(int32_t)), "malloc");
    check(hipMalloc(&xh, 2 * 4096 * sizeof(double)), "malloc");
    check(hipMemcpy(b0, T.data(), bytes, hipMemcpyHostToDevice), "h2d");
    check(hipMemset(b1, 0, bytes), "memset");
    check(smx_reset(b0, &sh, 0, 1, ctl, nullptr), "reset");
    check(smx_run(b0, b1, &sh, 0, K, ctl, parts, log, xh, 4096, nullptr), "run");
    check(hipDeviceSynchronize(), "sync");
    static unsigned long long tr[2][kTraceBlocks][4];
    check(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_trace), sizeof(tr)), "trace");
    int grid = 0;
    for (int b = 0; b < kTraceBlocks; ++b)
        if (tr[0][b][0] || tr[1][b][0]) grid = b + 1;
    const int la = sh.nparts;
    // the last two launches: parity (K-1)&1 is the last, K&1 the one before
    for (int q = 0; q < 2; ++q) {
        const int p = (K - 2 + q) & 1;
        unsigned long long t0 = ~0ull, e_max = 0, d_max = 0, l_max = 0, s_max = 0;
        std::vector<double> dec, sw;
        for (int b = 0; b < grid; ++b) {
            if (!tr[p][b][0]) continue;
            t0 = std::min(t0, tr[p][b][0]);
        }
        for (int b = 0; b < grid; ++b) {
            const auto* t = tr[p][b];
            if (!t[0]) continue;
            e_max = std::max(e_max, t[0] - t0);
            d_max = std::max(d_max, t[1] - t0);
            dec.push_back((t[1] - t0) / 100.0);
            if (b < la && t[2]) l_max = std::max(l_max, t[2] - t0);
            if (t[3]) {
                s_max = std::max(s_max, t[3] - t0);
                sw.push_back((t[3] - t0) / 100.0);
            }
        }
        std::sort(dec.begin(), dec.end());
        std::sort(sw.begin(), sw.end());
        printf("{\"size\":%d,\"launch\":%d,\"blocks\":%d,\"la_blocks\":%d,"
               "\"entry_spread_us\":%.2f,\"decision_median_us\":%.2f,\"decision_max_us\":%.2f,"
               "\"lookahead_done_max_us\":%.2f,\"sweep_done_median_us\":%.2f,"
               "\"sweep_done_max_us\":%.2f,\"start_tick\":%llu,\"end_tick\":%llu}\n",
               S, q, grid, la, e_max / 100.0, dec.empty() ? 0 : dec[dec.size() / 2],
               d_max / 100.0, l_max / 100.0, sw.empty() ? 0 : sw[sw.size() / 2], s_max / 100.0,
               t0, t0 + std::max(s_max, l_max));
    }
    return 0;
}
