// smx_host.hpp -- the host engine: pick_element and recalculate_matrix on a HOST tableau, for
// machines without an MI355X (the reference UI's 2-variable LPs, BASELINE config 1).
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
//
// Same layout and outcome codes as the device engine (row-major fp64, R = n+1 rows, leading
// dimension ld, f-row entries j >= flen are padding), same decisions and the same per-element
// expression, so a host tableau and a device tableau walk bit-identical trajectories:
//   selection   simplex.py:72-91 (phase 1), :93-103 (entering column / optimum), :105-141 (ratio
//               test as the key arg-min of smx_common.hpp, a NaN first candidate sticking);
//   update      simplex.py:149-177: out = num / e with num = -x (pivot row), x (pivot column),
//               1 (pivot element), x*e - pr*pc (all others), each operation rounded on its own
//               (-ffp-contract=off and the pragma below: no FMA).
#pragma once
#pragma clang fp contract(off)

namespace {

struct HostCand {
    int cls;   // 0: v < 0, 1: v == 0 (incl. -0.0), 2: v > 0, 3: none
    int idx;
    double v;
};

inline bool host_better(const HostCand& a, const HostCand& b) {
    if (a.cls != b.cls) return a.cls < b.cls;
    if (a.cls == 0) return (a.v > b.v) || (a.v == b.v && a.idx > b.idx);
    return a.idx < b.idx;
}

// pick_element on a host tableau: returns the SMX_* status, writes (r, c) when it pivots.
int host_select(const double* T, int64_t ld, int n, int m, int flen, int* r_out, int* c_out) {
    *r_out = SMX_NONE;
    *c_out = SMX_NONE;
    for (int i = 0; i < n; ++i) {                       // simplex.py:73-76
        if (T[(int64_t)i * ld + m] < 0.0) {
            const double* row = T + (int64_t)i * ld;
            *r_out = i;
            for (int j = 0; j < m; ++j) {               // simplex.py:82-85
                if (row[j] > 0.0) {
                    *c_out = j;
                    return SMX_PIVOT;
                }
            }
            return SMX_INCORRECT;                       // simplex.py:88-89
        }
    }
    const double* f = T + (int64_t)n * ld;
    const int fscan = flen < m ? flen : m;
    int c = SMX_NONE;
    for (int j = 0; j < fscan; ++j) {                   // simplex.py:94-98
        if (f[j] < 0.0) {
            c = j;
            break;
        }
    }
    if (c == SMX_NONE) return (flen < m) ? SMX_FSHORT : SMX_OPTIMUM;   // :95-96, :101-103
    *c_out = c;
    int first = SMX_NONE;
    double first_v = 0.0;
    HostCand best{3, SMX_NONE, 0.0};
    for (int i = 0; i < n; ++i) {                       // simplex.py:111-136
        const double a = T[(int64_t)i * ld + c];
        if (a != 0.0) {                                 // :112 (a NaN entry counts)
            const double v = T[(int64_t)i * ld + m] / a;   // :115
            if (first == SMX_NONE) {
                first = i;
                first_v = v;
            }
            if (!__builtin_isnan(v)) {
                HostCand x{(v < 0.0) ? 0 : ((v == 0.0) ? 1 : 2), i, v};
                if (host_better(x, best)) best = x;
            }
        }
    }
    if (first == SMX_NONE) return SMX_NOT_CONVERGE;     // :138-139
    if (__builtin_isnan(first_v)) {                     // :117-121
        *r_out = first;
        return SMX_PIVOT;
    }
    if (best.cls >= 2) return SMX_NOT_CONVERGE;
    *r_out = best.idx;
    return SMX_PIVOT;
}

// recalculate_matrix (simplex.py:149-177), out of place: every element of rows 0..n, columns
// 0..C-1 of Tout from Tin.
void host_pivot(const double* Tin, double* Tout, int64_t ld, int R, int C, int r, int c) {
    const double e = Tin[(int64_t)r * ld + c];
    const double* pr = Tin + (int64_t)r * ld;
    for (int i = 0; i < R; ++i) {
        const double* x = Tin + (int64_t)i * ld;
        double* o = Tout + (int64_t)i * ld;
        if (i == r) {
            for (int j = 0; j < C; ++j) o[j] = -x[j] / e;     // step 1 (:155-156)
            o[c] = 1.0 / e;                                   // step 3 (:163)
            continue;
        }
        const double pc = x[c];
        for (int j = 0; j < C; ++j) o[j] = (x[j] * e - pr[j] * pc) / e;   // step 4 (:166-175)
        o[c] = pc / e;                                        // step 2 (:159-160)
    }
}

}  // namespace

extern "C" {

int smx_host_select(const double* T, const smx_shape* s, int32_t* rc_out) {
    int r, c;
    const int st = host_select(T, s->ld, s->n, s->m, s->flen, &r, &c);
    rc_out[0] = r;
    rc_out[1] = c;
    return st;
}

int smx_host_pivot(const double* Tin, double* Tout, const smx_shape* s, int32_t r, int32_t c) {
    if (r < 0 || r > s->n || c < 0 || c > s->m) return -1;
    host_pivot(Tin, Tout, s->ld, s->n + 1, s->m + 1, r, c);
    return 0;
}

int64_t smx_host_run(double* buf0, double* buf1, const smx_shape* s, int32_t parity, int64_t k,
                     int32_t* log, int32_t* status_out) {
    double* buf[2] = {buf0, buf1};
    int64_t done = 0;
    int st = SMX_PIVOT;
    while (done < k) {
        int r, c;
        const double* T = buf[(parity + done) & 1];
        st = host_select(T, s->ld, s->n, s->m, s->flen, &r, &c);
        if (st != SMX_PIVOT) break;
        if (s->flen > s->m + 1 || (s->flen < s->m && c >= s->flen)) {
            st = SMX_FSHORT;   // the reference indexes the f-row out of range (simplex.py:159-175)
            break;
        }
        host_pivot(T, buf[(parity + done + 1) & 1], s->ld, s->n + 1, s->m + 1, r, c);
        if (log) {
            log[2 * done] = r;
            log[2 * done + 1] = c;
        }
        ++done;
    }
    *status_out = (done == k && st == SMX_PIVOT) ? SMX_IDLE : st;
    return done;
}

}  // extern "C"
