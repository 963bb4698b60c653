/*
 * CPU ORACLE (test infrastructure only) -- C restatement of the reference pivot loop.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library
 * (oracle/_build/libsmx_oracle.so), as the checker or as the timed CPU baseline; the product
 * path never links it.
 *
 * Restates /root/reference/src/simplex.py (jqnfxa/Simplex-Method-Solver @ 2025-06-20) on a
 * dense row-major fp64 tableau T[R][ld] (R = n+1 rows incl. the f-row, C = m+1 columns):
 *   smx_oracle_pick  <- SimplexMethod.pick_element      simplex.py:70-141
 *   smx_oracle_pivot <- SimplexMethod.recalculate_matrix simplex.py:143-177 (steps 1-4)
 *   smx_oracle_run   <- the loop of get_solution         simplex.py:184-198 (no snapshots)
 * Compiled with -ffp-contract=off: t*e, pr*pc, the subtraction and the division are each
 * rounded, exactly like CPython floats.  Pinned against the reference's fixtures by
 * tests/test_oracle_golden.py.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define ST_PIVOT 0
#define ST_OPTIMUM 1
#define ST_INCORRECT 2
#define ST_NOT_CONVERGE 3
#define ST_FSHORT 4

/* pick_element: phase 1 (simplex.py:72-91), entering column (:94-103), ratio test (:105-141). */
int smx_oracle_pick(const double* T, int64_t ld, int32_t n, int32_t m, int32_t flen,
                    int32_t* r_out, int32_t* c_out) {
    *r_out = -1;
    *c_out = -1;
    for (int32_t i = 0; i < n; ++i) {
        if (T[(int64_t)i * ld + m] < 0) {
            *r_out = i;
            for (int32_t j = 0; j < m; ++j) {
                if (T[(int64_t)i * ld + j] > 0) {
                    *c_out = j;
                    return ST_PIVOT;
                }
            }
            return ST_INCORRECT;
        }
    }
    const double* f = T + (int64_t)n * ld;
    int32_t scan = m < flen ? m : flen;
    int32_t c = -1;
    for (int32_t j = 0; j < scan; ++j) {
        if (f[j] < 0) {
            c = j;
            break;
        }
    }
    if (c < 0) return flen < m ? ST_FSHORT : ST_OPTIMUM;
    *c_out = c;
    /* the reference's state machine, sequential form (simplex.py:107-136) */
    int32_t best = -1;
    double bv = 1.0;
    for (int32_t i = 0; i < n; ++i) {
        double a = T[(int64_t)i * ld + c];
        if (a == 0) continue;
        double v = T[(int64_t)i * ld + m] / a;
        if (best < 0) {
            best = i;
            bv = v;
        } else if (v == 0 && bv > 0) {
            best = i;
            bv = v;
        } else if (v < 0 && 0 <= bv) {
            best = i;
            bv = v;
        } else if (bv <= v && v < 0) {
            best = i;
            bv = v;
        }
    }
    if (best < 0 || bv > 0) return ST_NOT_CONVERGE;
    *r_out = best;
    return ST_PIVOT;
}

/* recalculate_matrix steps 1-4 (simplex.py:155-175), out of place, all reads from Tin. */
void smx_oracle_pivot(const double* Tin, double* Tout, int64_t ld, int32_t R, int32_t C,
                      int32_t r, int32_t c, int32_t nthreads) {
    const double e = Tin[(int64_t)r * ld + c];
    const double* pr = Tin + (int64_t)r * ld;
    (void)nthreads;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int32_t i = 0; i < R; ++i) {
        const double* src = Tin + (int64_t)i * ld;
        double* dst = Tout + (int64_t)i * ld;
        const double pc = src[c];
        if (i == r) {
            for (int32_t j = 0; j < C; ++j) dst[j] = -src[j] / e;
            dst[c] = 1.0 / e;
        } else {
            for (int32_t j = 0; j < C; ++j) {
                double a = src[j] * e;
                double b = pr[j] * pc;
                dst[j] = (a - b) / e;
            }
            dst[c] = pc / e;
        }
    }
}

/* get_solution's loop without snapshots; ping-pong between A and B.  Returns pivots done;
 * *which = 0 if the final table is in A, 1 if in B. */
int64_t smx_oracle_run(double* A, double* B, int64_t ld, int32_t n, int32_t m, int32_t flen,
                       int64_t max_pivots, int32_t* log_rc, int32_t* which, int32_t* status,
                       int32_t nthreads) {
    double* cur = A;
    double* nxt = B;
    int64_t done = 0;
    *status = ST_PIVOT;
    while (done < max_pivots) {
        int32_t r, c;
        int st = smx_oracle_pick(cur, ld, n, m, flen, &r, &c);
        if (st != ST_PIVOT) {
            *status = st;
            break;
        }
        if (log_rc) {
            log_rc[2 * done] = r;
            log_rc[2 * done + 1] = c;
        }
        smx_oracle_pivot(cur, nxt, ld, n + 1, m + 1, r, c, nthreads);
        double* t = cur;
        cur = nxt;
        nxt = t;
        ++done;
    }
    *which = (cur == A) ? 0 : 1;
    return done;
}
