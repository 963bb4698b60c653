// smx_intfirst.hpp -- the first pivot of a tableau given as Python ints (simplex.py:155-175 on
// int operands), on the device and on the host.
// Part of libsmx (compiled as one translation unit by smx_kernels.hip; not a standalone header).
//
// The reference keeps the caller's numbers as they come (simplex.py:36-39), so an int entry stays
// an int until the first recalculate_matrix writes every element through `/` (float from then on).
// On that one pivot, with |ints| < 2^26 (every product and difference exact in fp64), the int
// arithmetic and the fp64 one agree in every bit EXCEPT the sign of a zero:
//   pivot row     -t / e:              t an int 0: -0 is the int 0, so 0 / e has e's sign; fp64's
//                                      -(+0.0) / e has the opposite one;
//   other entries (t*e - pr*pc) / e:   an int*int product that is 0 is the int 0 (+0.0 once mixed
//                                      with a float), where fp64's 0.0 * -3.0 is -0.0 -- and a
//                                      zero numerator carries that sign into the quotient;
//   pivot column t / e and the pivot 1.0 / e: identical.
// So after the regular fp64 pivot (any engine) only the entries that came out +-0 can be wrong,
// and they are recomputed here with each int*int product's zero made +0 (an int numerator of 0 is
// +0 - +0 = +0 in fp64 too).  `mask` marks the int entries of T0 (NULL: every entry is an int);
// `maskr` is the pivot row's mask (the row may live on another rank: `prow` is T0's pivot row).
// Pinned against the reference run on int and mixed int / float inputs (tests/golden/intzero.json).

namespace {

__device__ __host__ __forceinline__ double int_first_value(double t, double e, double pr,
                                                           double pc, bool rowr, bool mij,
                                                           bool mrc, bool mrj, bool mic) {
    if (rowr) return ((mij && t == 0.0) ? 0.0 : -t) / e;   // simplex.py:155-156 (-0 is int 0)
    double a = t * e;                                      // simplex.py:173-175
    double b = pr * pc;
    if (mij && mrc && a == 0.0) a = 0.0;                   // int * int == 0: the int 0
    if (mrj && mic && b == 0.0) b = 0.0;
    return (a - b) / e;
}

// One workgroup per row (grid-stride over rows), lanes over columns: reads T1, and T0 / prow /
// the masks only where T1 holds a zero.
__global__ __launch_bounds__(256) void k_int_first_fix(const double* __restrict__ T0,
                                                       double* __restrict__ T1, int64_t ld,
                                                       int rows, int C, int r_local, int c,
                                                       const double* __restrict__ prow,
                                                       const uint8_t* __restrict__ mask,
                                                       int64_t ldm,
                                                       const uint8_t* __restrict__ maskr) {
    const double e = prow[c];
    const bool mrc = maskr ? maskr[c] != 0 : true;
    for (int i = blockIdx.x; i < rows; i += gridDim.x) {
        const double* t0 = T0 + (int64_t)i * ld;
        double* t1 = T1 + (int64_t)i * ld;
        const uint8_t* mi = mask ? mask + (int64_t)i * ldm : nullptr;
        const bool rowr = i == r_local;
        for (int j = threadIdx.x; j < C; j += blockDim.x) {
            if (j == c || t1[j] != 0.0) continue;   // pivot column / element: no difference
            const bool mij = mi ? mi[j] != 0 : true;
            const bool mic = mi ? mi[c] != 0 : true;
            const bool mrj = maskr ? maskr[j] != 0 : true;
            t1[j] = int_first_value(t0[j], e, prow[j], t0[c], rowr, mij, mrc, mrj, mic);
        }
    }
}

void host_int_first_fix(const double* T0, double* T1, int64_t ld, int rows, int C, int r_local,
                        int c, const double* prow, const uint8_t* mask, int64_t ldm,
                        const uint8_t* maskr) {
    const double e = prow[c];
    const bool mrc = maskr ? maskr[c] != 0 : true;
    for (int i = 0; i < rows; ++i) {
        const double* t0 = T0 + (int64_t)i * ld;
        double* t1 = T1 + (int64_t)i * ld;
        const uint8_t* mi = mask ? mask + (int64_t)i * ldm : nullptr;
        for (int j = 0; j < C; ++j) {
            if (j == c || t1[j] != 0.0) continue;
            const bool mij = mi ? mi[j] != 0 : true;
            const bool mic = mi ? mi[c] != 0 : true;
            const bool mrj = maskr ? maskr[j] != 0 : true;
            t1[j] = int_first_value(t0[j], e, prow[j], t0[c], i == r_local, mij, mrc, mrj, mic);
        }
    }
}

bool int_first_args_ok(const double* T0, const double* T1, int64_t ld, int rows, int C,
                       int r_local, int c, const double* prow, const uint8_t* mask, int64_t ldm) {
    return T0 && T1 && prow && T0 != T1 && rows >= 1 && C >= 1 && ld >= C && c >= 0 && c < C &&
           r_local >= -1 && r_local < rows && (!mask || ldm >= C);
}

}  // namespace
