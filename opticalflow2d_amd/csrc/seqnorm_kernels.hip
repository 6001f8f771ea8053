// seqnorm_kernels.hip — the reference's Logger norms, bit for bit.
//
// Motion::norm (src/Motion.cpp:42-49) adds the N pixel magnitudes
//   d_k = sqrt((double)x_k^2 + (double)y_k^2)     (std::pow(float, 2) is double)
// to a FLOAT running sum in linear index order (idx = i + j*dimx,
// src/Field.tpp:13):
//   S <- (float)((double)S + d_k)
// and returns S / (float)N; Logger::update_error (src/Logger.cpp:32-51) takes
// it of (motion - prev) and of prev.  At 4096^2 the rounding of that sum moves
// the error 2-6 % away from the exactly summed one, and with it the iteration
// at which ImageRegistrationOpticalFlow.cpp:131-134 breaks, so the default
// Logger mode computes the float running sum itself.
//
// Parallel form.  While S stays inside one binade
// [2^e, 2^(e+1)) its ulp is u = 2^(e-23) and S = M u, M in [2^23, 2^24).  The
// double sum S + d_k rounds d_k to the grid 2^(e-52) (S is an even multiple of
// that grid, so ties-to-even depends on d_k alone); the float rounding then
// adds an integer m_k(e) of ulps that depends on d_k and e only, unless the
// rounded d_k lies exactly halfway between two ulps (a tie, whose direction
// depends on the parity of M).  So while M plus the running sum of m_k(e)
// stays <= 2^24 - 1 (no binade crossing) and no tie occurs, S after a run of
// terms is (M + sum m_k(e)) u exactly: an integer prefix sum.  Crossings (a
// few dozen per norm: S doubles between them) and ties are stepped one term
// at a time with the reference's own two roundings.
//
// Pipeline for the pair of norms of one Logger update (|cur - prev| and
// |prev|), in tiles of kSnTile consecutive terms:
//   seqnorm_tile_sums    fp64 sum of each tile's magnitudes (a prediction)
//   seqnorm_candidates   fp64 prefix over the tiles -> per tile the <= 4
//                        binades the running sum can lie in across the tile
//   seqnorm_tables       per tile and candidate binade: sum of m_k(e) and a
//                        tie / NaN flag
//   seqnorm_walk         one block per norm walks the tiles in order, 1024
//                        tiles per step (saturating block scan of their table
//                        entries for the current binade); a tile whose entry
//                        does not apply (a crossing, a tie, a binade outside
//                        its candidates) is resolved from its magnitudes.
// The prediction only decides how much resolving is needed: the walk's result
// is the reference's float sum whatever it predicted.
#include <hip/hip_runtime.h>

#include <cmath>

#include "of2d_device.h"

namespace of2d {
namespace {

constexpr int kSnThreads = 256;        // tile kernels
constexpr int kSnPerThread = kSnTile / kSnThreads;
constexpr int kSnWalk = 1024;          // walk block: tiles per step, terms / 4 per resolve
constexpr int kSnTerms = kSnTile / kSnWalk;
constexpr int kSnCand = 4;            // candidate binades per tile
constexpr int kSnEmin = -100;          // below 2^-100 the sum is "low": stepped per nonzero term
constexpr int kSnLow = -1000;
constexpr int kSnNonfinite = 1000;
constexpr unsigned kSnSat = 1u << 25;           // saturated sum of m: certainly a crossing
constexpr unsigned kSnLimit = (1u << 24) - 1u;  // largest M + sum that stays in the binade
constexpr unsigned kSnBad = 1u << 31;           // table entry: a tie or NaN among the terms
// header word of a tile / norm (seqnorm_candidates)
constexpr unsigned kHdrZero = 1u << 30;  // every magnitude of the tile is 0: a no-op
constexpr unsigned kHdrNan = 1u << 29;   // a NaN magnitude
__host__ __device__ constexpr unsigned hdr_pack(int elo, int nc) {
    return (unsigned)(elo + 512) | ((unsigned)nc << 16);
}
__device__ __forceinline__ int hdr_elo(unsigned h) { return (int)(h & 0xffffu) - 512; }
__device__ __forceinline__ int hdr_nc(unsigned h) { return (int)((h >> 16) & 7u); }

// binade of the running sum (S >= 0 or NaN)
__device__ __forceinline__ int sn_region(float S) {
    const unsigned ex = (__float_as_uint(S) >> 23) & 0xffu;
    if (ex == 0xffu) return kSnNonfinite;
    const int e = (int)ex - 127;
    return e < kSnEmin ? kSnLow : e;
}
__device__ __forceinline__ unsigned sn_mant(float S) {
    return (__float_as_uint(S) & 0x7fffffu) | 0x800000u;
}
// the float (M + s) ulps in binade e, M + s <= kSnLimit
__device__ __forceinline__ float sn_make(int e, unsigned M) {
    return __uint_as_float(((unsigned)(e + 127) << 23) | (M - 0x800000u));
}
__device__ __forceinline__ unsigned sn_sat(unsigned a, unsigned b) {
    const unsigned s = a + b;  // a, b <= kSnSat
    return s < kSnSat ? s : kSnSat;
}
// Motion::norm's magnitude: float components squared and added in double
// (-ffp-contract=off: no fused multiply-add), double sqrt (correctly rounded)
__device__ __forceinline__ double sn_mag(float x, float y) {
    const double a = x, b = y;
    return sqrt(a * a + b * b);
}
// ulps that (float)((double)S + d) adds to S = M 2^(e-23) while the result
// stays in the binade; `bad` on a tie (parity-dependent) or NaN.  scale =
// 2^(52-e): d * scale is exact, rint rounds it to the double sum's grid
// (ties to even: S / grid is even), and the float rounding of the rest to an
// integer number of ulps (2^29 grid units) is exact arithmetic on doubles.
__device__ __forceinline__ unsigned sn_incr(double d, double scale, bool &bad) {
    const double x = d * scale;
    if (!(x < 9007199254740992.0)) {  // d >= 2^(e+1): crosses; or NaN
        bad |= (x != x);
        return kSnSat;
    }
    const double t = rint(x) * 0x1p-29;
    const double m0 = floor(t);
    const double fr = t - m0;
    bad |= (fr == 0.5);
    return (unsigned)m0 + (fr > 0.5 ? 1u : 0u);
}
__device__ __forceinline__ double sn_scale(int e) {
    return __longlong_as_double((long long)(52 - e + 1023) << 52);
}

// The tile's terms of thread `tid`: kSnPerThread terms, strided by the block
// (term t = r * kSnThreads + tid), so a wave reads 64 consecutive pixels.
__device__ __forceinline__ void sn_tile_terms(const float2 *__restrict__ cur,
                                              const float2 *__restrict__ prev, unsigned base,
                                              unsigned N, int dimx, int P, double *dd,
                                              double *dp) {
    unsigned L = base + threadIdx.x;
    unsigned j = L / (unsigned)dimx, i = L - j * (unsigned)dimx;
#pragma unroll
    for (int r = 0; r < kSnPerThread; r++) {
        if (L < N) {
            const size_t off = (size_t)j * (size_t)P + i;
            const float2 c = cur[off], p = prev[off];
            dd[r] = sn_mag(c.x - p.x, c.y - p.y);  // Field::operator- (Field.tpp:305-334)
            dp[r] = sn_mag(p.x, p.y);
        } else {
            dd[r] = 0.0;
            dp[r] = 0.0;
        }
        L += kSnThreads;
        i += kSnThreads;
        while (i >= (unsigned)dimx) {
            i -= (unsigned)dimx;
            j++;
        }
    }
}

template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
    return v;
}

// ---------------------------------------------------------------- kernels
__global__ __launch_bounds__(kSnThreads) void seqnorm_tile_sums(const float2 *__restrict__ cur,
                                                               const float2 *__restrict__ prev,
                                                               unsigned N, int dimx, int P,
                                                               double *__restrict__ A) {
    double dd[kSnPerThread], dp[kSnPerThread];
    sn_tile_terms(cur, prev, blockIdx.x * (unsigned)kSnTile, N, dimx, P, dd, dp);
    double sd = 0.0, sp = 0.0;
#pragma unroll
    for (int r = 0; r < kSnPerThread; r++) {
        sd += dd[r];
        sp += dp[r];
    }
    auto add = [](double a, double b) { return a + b; };
    sd = wave_reduce(sd, add);
    sp = wave_reduce(sp, add);
    __shared__ double ws[2][kSnThreads / 64];
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        ws[0][w] = sd;
        ws[1][w] = sp;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        double s = 0.0;
        for (int k = 0; k < kSnThreads / 64; k++) s += ws[threadIdx.x][k];
        A[2 * (size_t)blockIdx.x + threadIdx.x] = s;
    }
}

// binade of a double bound, clamped to the float range
__device__ __forceinline__ int sn_region_d(double v) {
    if (!(v >= 0x1p-100)) return kSnLow;
    if (v >= 0x1p127) return 127;
    int ex;
    (void)frexp(v, &ex);
    return ex - 1;
}

__global__ __launch_bounds__(kSnWalk) void seqnorm_candidates(const double *__restrict__ A,
                                                              unsigned ntiles,
                                                              unsigned *__restrict__ H) {
    const unsigned chunk = (ntiles + kSnWalk - 1) / kSnWalk;
    const unsigned b0 = threadIdx.x * chunk;
    const unsigned b1 = min(ntiles, b0 + chunk);
    __shared__ double sh[2][kSnWalk];
    for (int n = 0; n < 2; n++) {
        double s = 0.0;
        for (unsigned b = b0; b < b1; b++) s += A[2 * (size_t)b + n];
        sh[n][threadIdx.x] = s;
    }
    __syncthreads();
    // exclusive prefix of the chunk sums (Hillis-Steele on LDS; a prediction, any order)
    for (int o = 1; o < kSnWalk; o <<= 1) {
        double v0 = 0.0, v1 = 0.0;
        if ((int)threadIdx.x >= o) {
            v0 = sh[0][threadIdx.x - o];
            v1 = sh[1][threadIdx.x - o];
        }
        __syncthreads();
        sh[0][threadIdx.x] += v0;
        sh[1][threadIdx.x] += v1;
        __syncthreads();
    }
    for (int n = 0; n < 2; n++) {
        double Pb = threadIdx.x ? sh[n][threadIdx.x - 1] : 0.0;
        for (unsigned b = b0; b < b1; b++) {
            const double a = A[2 * (size_t)b + n];
            unsigned h;
            if (a == 0.0) {
                h = kHdrZero;
            } else if (!(a < INFINITY) || !(Pb < INFINITY)) {
                h = hdr_pack(0, 0) | (a != a ? kHdrNan : 0u);
            } else {
                // the float sum's drift from the fp64 one stays within a few %
                // at the grid sizes the break test sees; 1/8 either side
                const int ehi = sn_region_d((Pb + a) * 1.125);
                int elo = sn_region_d(Pb * 0.875);
                if (elo == kSnLow) elo = kSnEmin;
                if (ehi == kSnLow) {
                    h = hdr_pack(0, 0);
                } else {
                    if (ehi - elo + 1 > kSnCand) elo = ehi - kSnCand + 1;
                    h = hdr_pack(elo, ehi - elo + 1);
                }
            }
            H[2 * (size_t)b + n] = h;
            Pb += a;
        }
    }
}

__global__ __launch_bounds__(kSnThreads) void seqnorm_tables(const float2 *__restrict__ cur,
                                                            const float2 *__restrict__ prev,
                                                            unsigned N, int dimx, int P,
                                                            const unsigned *__restrict__ H,
                                                            unsigned *__restrict__ T) {
    const unsigned h0 = H[2 * (size_t)blockIdx.x], h1 = H[2 * (size_t)blockIdx.x + 1];
    if (hdr_nc(h0) == 0 && hdr_nc(h1) == 0) return;
    double dd[kSnPerThread], dp[kSnPerThread];
    sn_tile_terms(cur, prev, blockIdx.x * (unsigned)kSnTile, N, dimx, P, dd, dp);
    __shared__ unsigned ws[2][kSnCand][kSnThreads / 64];
    const int w = threadIdx.x / 64;
    auto sat = [](unsigned a, unsigned b) {
        return ((a | b) & kSnBad) | sn_sat(a & ~kSnBad, b & ~kSnBad);
    };
    for (int n = 0; n < 2; n++) {
        const unsigned h = n ? h1 : h0;
        const int nc = hdr_nc(h), elo = hdr_elo(h);
        for (int c = 0; c < nc; c++) {
            const double scale = sn_scale(elo + c);
            unsigned s = 0;
            bool bad = false;
#pragma unroll
            for (int r = 0; r < kSnPerThread; r++)
                s = sn_sat(s, sn_incr(n ? dp[r] : dd[r], scale, bad));
            s = wave_reduce(s | (bad ? kSnBad : 0u), sat);
            if ((threadIdx.x & 63) == 0) ws[n][c][w] = s;
        }
    }
    __syncthreads();
    if (threadIdx.x < 2 * kSnCand) {
        const int n = threadIdx.x / kSnCand, c = threadIdx.x % kSnCand;
        if (c < hdr_nc(n ? h1 : h0)) {
            unsigned s = ws[n][c][0];
            for (int k = 1; k < kSnThreads / 64; k++) s = sat(s, ws[n][c][k]);
            T[(2 * (size_t)blockIdx.x + n) * kSnCand + c] = s;
        }
    }
}

// ---------------------------------------------------------------- the walk
// A run of terms inside one binade as a function of the parity of M:
// M -> M + (M even ? lo : hi), packed lo | hi << 32.  A term without a tie
// adds m ulps either way; a tie (d rounded to exactly m0 + 1/2 ulps) rounds
// M + m0 + 1/2 to even, i.e. adds m0 or m0 + 1 by the parity of M.  The form
// is closed under composition, so the walk's resolves scan ties like any other
// term (a constant field of dyadic magnitudes ties on every term).
typedef unsigned long long sn_fn;
__device__ __forceinline__ sn_fn fn_make(unsigned e, unsigned o) {
    return (sn_fn)e | ((sn_fn)o << 32);
}
__device__ __forceinline__ unsigned fn_e(sn_fn f) { return (unsigned)f; }
__device__ __forceinline__ unsigned fn_o(sn_fn f) { return (unsigned)(f >> 32); }
// g after f
__device__ __forceinline__ sn_fn fn_then(sn_fn f, sn_fn g) {
    const unsigned fe = fn_e(f), fo = fn_o(f);
    return fn_make(sn_sat(fe, (fe & 1u) ? fn_o(g) : fn_e(g)),
                   sn_sat(fo, (fo & 1u) ? fn_e(g) : fn_o(g)));
}
__device__ __forceinline__ unsigned fn_apply(sn_fn f, unsigned M) {
    return M + ((M & 1u) ? fn_o(f) : fn_e(f));
}
// the term's function in binade `scale`; `nan` for a NaN magnitude
__device__ __forceinline__ sn_fn sn_term_fn(double d, double scale, bool &nan) {
    const double x = d * scale;
    if (!(x < 9007199254740992.0)) {
        nan |= (x != x);
        return fn_make(kSnSat, kSnSat);
    }
    const double t = rint(x) * 0x1p-29;
    const double m0d = floor(t);
    const double fr = t - m0d;
    const unsigned m0 = (unsigned)m0d;
    if (fr == 0.5) return fn_make(m0 + (m0 & 1u), m0 + ((m0 + 1u) & 1u));
    const unsigned m = m0 + (fr > 0.5 ? 1u : 0u);
    return fn_make(m, m);
}

// block-wide primitives of the 1024-thread walk block
struct WalkShared {
    unsigned wsum[kSnWalk / 64];
    unsigned wmin[kSnWalk / 64];
    sn_fn wfn[kSnWalk / 64];
    unsigned base;  // exclusive prefix at the first failing tile
    float S;
};

__device__ __forceinline__ unsigned wave_incl_sat(unsigned v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(v, o, 64);
        if (lane >= o) v = sn_sat(v, t);
    }
    return v;
}
// saturating scan over the block in thread order: returns the inclusive
// prefix, *excl the exclusive one (both exact while below kSnSat), *total the
// block total
__device__ unsigned block_scan_sat(unsigned v, WalkShared &sh, unsigned *excl, unsigned *total) {
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    const unsigned wi = wave_incl_sat(v);
    unsigned we = __shfl_up(wi, 1, 64);
    if (lane == 0) we = 0;
    if (lane == 63) sh.wsum[w] = wi;
    __syncthreads();
    unsigned pre = 0, tot = 0;
    for (int k = 0; k < kSnWalk / 64; k++) {
        if (k < w) pre = sn_sat(pre, sh.wsum[k]);
        tot = sn_sat(tot, sh.wsum[k]);
    }
    __syncthreads();
    *total = tot;
    *excl = sn_sat(pre, we);
    return sn_sat(pre, wi);
}
// ordered scan of functions: *excl = composition of the earlier threads'
// functions, returns the composition over the whole block
__device__ sn_fn block_scan_fn(sn_fn v, WalkShared &sh, sn_fn *excl) {
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const sn_fn t = __shfl_up(v, o, 64);
        if (lane >= o) v = fn_then(t, v);
    }
    sn_fn we = __shfl_up(v, 1, 64);
    if (lane == 0) we = 0;
    if (lane == 63) sh.wfn[w] = v;
    __syncthreads();
    sn_fn pre = 0, tot = 0;
    for (int k = 0; k < kSnWalk / 64; k++) {
        if (k < w) pre = fn_then(pre, sh.wfn[k]);
        tot = fn_then(tot, sh.wfn[k]);
    }
    __syncthreads();
    *excl = fn_then(pre, we);
    return tot;
}
__device__ unsigned block_min(unsigned v, WalkShared &sh) {
    const int w = threadIdx.x / 64;
    v = wave_reduce(v, [](unsigned a, unsigned b) { return a < b ? a : b; });
    if ((threadIdx.x & 63) == 0) sh.wmin[w] = v;
    __syncthreads();
    unsigned m = sh.wmin[0];
    for (int k = 1; k < kSnWalk / 64; k++) m = min(m, sh.wmin[k]);
    __syncthreads();
    return m;
}
__device__ bool block_any(bool v, WalkShared &sh) { return block_min(v ? 0u : 1u, sh) == 0u; }

// Tile `tile` from the exact running sum S: thread tid holds terms
// [kSnTerms tid, kSnTerms (tid + 1)) of the tile.  Each round takes the binade
// of S, composes the terms after `pos` by an ordered block scan up to the first
// term that leaves the binade, is NaN, or (low sum) is nonzero, and steps that
// one term as the reference does.
__device__ float sn_resolve(const float2 *__restrict__ cur, const float2 *__restrict__ prev,
                            int which, unsigned tile, unsigned N, int dimx, int P, float S,
                            WalkShared &sh) {
    double d[kSnTerms];
    {
        const unsigned L = tile * (unsigned)kSnTile + kSnTerms * threadIdx.x;
        unsigned j = L / (unsigned)dimx, i = L - j * (unsigned)dimx;
#pragma unroll
        for (int k = 0; k < kSnTerms; k++) {
            d[k] = 0.0;
            if (L + k < N) {
                const size_t off = (size_t)j * (size_t)P + i;
                const float2 p = prev[off];
                if (which == 0) {
                    const float2 c = cur[off];
                    d[k] = sn_mag(c.x - p.x, c.y - p.y);
                } else {
                    d[k] = sn_mag(p.x, p.y);
                }
            }
            if (++i == (unsigned)dimx) {
                i = 0;
                j++;
            }
        }
    }
    unsigned pos = 0;  // first term of the tile not yet added
    for (;;) {
        const int e = sn_region(S);
        if (e == kSnNonfinite) {
            bool nan = false;
#pragma unroll
            for (int k = 0; k < kSnTerms; k++)
                nan |= (kSnTerms * threadIdx.x + k >= pos) && (d[k] != d[k]);
            return block_any(nan, sh) ? __uint_as_float(0x7fc00000u) : S;
        }
        const bool low = (e == kSnLow);
        const unsigned M = low ? 0u : sn_mant(S);
        const double scale = low ? 0.0 : sn_scale(e);
        sn_fn f[kSnTerms], tf = 0;
        bool fail[kSnTerms];
#pragma unroll
        for (int k = 0; k < kSnTerms; k++) {
            bool bad = false;
            f[k] = 0;
            if (kSnTerms * threadIdx.x + k >= pos) {
                if (low)
                    bad = (d[k] != 0.0);  // NaN too
                else
                    f[k] = sn_term_fn(d[k], scale, bad);
            }
            fail[k] = bad;
            tf = fn_then(tf, f[k]);
        }
        sn_fn excl;
        const sn_fn tot = block_scan_fn(tf, sh, &excl);
        // this thread's first term that fails or takes M past the binade (the
        // running M is exact up to the block's first such term)
        unsigned R = fn_apply(excl, M), myfirst = 0xffffffffu, mybase = 0;
#pragma unroll
        for (int k = 0; k < kSnTerms; k++) {
            if (myfirst != 0xffffffffu) break;
            const unsigned nR = fn_apply(f[k], R);
            if (fail[k] || nR > kSnLimit) {
                myfirst = kSnTerms * threadIdx.x + k;
                mybase = R;
            } else {
                R = nR;
            }
        }
        const unsigned first = block_min(myfirst, sh);
        if (first == 0xffffffffu) return low ? S : sn_make(e, fn_apply(tot, M));
        if (myfirst == first) {
            const float Sf = low ? S : sn_make(e, mybase);
            sh.S = (float)((double)Sf + d[first - kSnTerms * threadIdx.x]);  // Motion.cpp:46
        }
        __syncthreads();
        S = sh.S;
        __syncthreads();
        pos = first + 1;
    }
}

__global__ __launch_bounds__(kSnWalk) void seqnorm_walk(const float2 *__restrict__ cur,
                                                        const float2 *__restrict__ prev,
                                                        unsigned N, int dimx, int P,
                                                        unsigned ntiles,
                                                        const unsigned *__restrict__ H,
                                                        const unsigned *__restrict__ T,
                                                        float *__restrict__ out,
                                                        int *__restrict__ dbg) {
    __shared__ WalkShared sh;
    const int n = blockIdx.x;  // 0: |cur - prev|, 1: |prev|
    float S = 0.0f;
    unsigned b = 0;
    int resolves = 0;
    bool nan = false;  // non-finite sum: a NaN magnitude after it
    while (b < ntiles) {
        const unsigned tb = b + threadIdx.x;
        const int e = sn_region(S);
        unsigned h = kHdrZero;
        if (tb < ntiles) h = H[2 * (size_t)tb + n];
        if (e == kSnNonfinite) {
            nan |= (h & kHdrNan) != 0;
            b += kSnWalk;
            continue;
        }
        unsigned v = 0;
        bool fail = false;
        if (!(h & kHdrZero)) {
            const int c = e - hdr_elo(h);
            if (e == kSnLow || c < 0 || c >= hdr_nc(h)) {
                fail = true;
            } else {
                const unsigned w = T[(2 * (size_t)tb + n) * kSnCand + c];
                fail = (w & kSnBad) != 0;
                v = w & ~kSnBad;
            }
        }
        const unsigned M = (e == kSnLow) ? 0u : sn_mant(S);
        unsigned total, excl;
        const unsigned incl = block_scan_sat(v, sh, &excl, &total);
        fail |= (M + incl > kSnLimit);
        const unsigned first = block_min(fail ? threadIdx.x : 0xffffffffu, sh);
        if (first == 0xffffffffu) {
            if (e != kSnLow) S = sn_make(e, M + total);  // low: all tiles were zero
            b += kSnWalk;
            continue;
        }
        if (threadIdx.x == first) sh.base = excl;  // exact: no earlier thread failed
        __syncthreads();
        if (e != kSnLow && first > 0) S = sn_make(e, M + sh.base);
        __syncthreads();
        S = sn_resolve(cur, prev, n, b + first, N, dimx, P, S, sh);
        resolves++;
        b += first + 1;
    }
    if (threadIdx.x == 0) {
        if (nan) S = __uint_as_float(0x7fc00000u);
        out[n] = S;
        if (dbg) dbg[n] = resolves;
    }
}

}  // namespace

size_t seqnorm_workspace_bytes(int dimx, int dimy) {
    const size_t N = (size_t)dimx * (size_t)dimy;
    const size_t nt = (N + kSnTile - 1) / kSnTile;
    return nt * (2 * sizeof(double) + 2 * sizeof(unsigned) + 2 * kSnCand * sizeof(unsigned));
}

void launch_seqnorm(const float2 *cur, const float2 *prev, int dimx, int dimy, int P, void *ws,
                    float *out, int *dbg, hipStream_t st) {
    const size_t N = (size_t)dimx * (size_t)dimy;
    if (dimx <= 0 || dimy <= 0 || P < dimx || N > 0xffffffffu)
        throw std::invalid_argument("launch_seqnorm: bad geometry");
    const unsigned nt = (unsigned)((N + kSnTile - 1) / kSnTile);
    double *A = static_cast<double *>(ws);
    unsigned *H = reinterpret_cast<unsigned *>(A + 2 * (size_t)nt);
    unsigned *T = H + 2 * (size_t)nt;
    hipLaunchKernelGGL(seqnorm_tile_sums, dim3(nt), dim3(kSnThreads), 0, st, cur, prev,
                       (unsigned)N, dimx, P, A);
    OF2D_HIP(hipGetLastError());
    hipLaunchKernelGGL(seqnorm_candidates, dim3(1), dim3(kSnWalk), 0, st, A, nt, H);
    OF2D_HIP(hipGetLastError());
    hipLaunchKernelGGL(seqnorm_tables, dim3(nt), dim3(kSnThreads), 0, st, cur, prev, (unsigned)N,
                       dimx, P, H, T);
    OF2D_HIP(hipGetLastError());
    hipLaunchKernelGGL(seqnorm_walk, dim3(2), dim3(kSnWalk), 0, st, cur, prev, (unsigned)N, dimx,
                       P, nt, H, T, out, dbg);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
