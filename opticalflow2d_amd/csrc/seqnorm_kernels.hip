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
// few dozen per norm: S doubles between them) are stepped one term at a time
// with the reference's own two roundings; inside the walk's term-level scans
// ties are composed exactly (a run of terms is M -> M + (M even ? a : b)).
//
// Pipeline (round 4).  The norms of a batch of K <= 3 consecutive Logger
// updates (a Jacobi triple's: pair i = iterates u[i], u[i + 1] on workspace
// ws[i]) run as one launch per stage, in tiles of kSnTile consecutive terms
// and segments of 64:
//   seqnorm_tables<K>   the pass: one wave per tile reads the K + 1 iterates
//                       once and writes per norm the fp64 tile sum (a
//                       prediction), the nonzero-segment mask, the header and,
//                       for the <= 2 binades the workspace's profile predicts
//                       (its last walk's running sums scaled by the trend of
//                       its totals), the tile entries: each lane adds its
//                       terms' ulp increments, decided from an fp32 estimate
//                       of the magnitude wherever it lies clear of a
//                       half-integer (sn_incr_est), the exact fp64 sequence in
//                       the waves where one lane's estimate does not decide
//   seqnorm_check       (three launches: block sums, scan, check) the fp64
//                       prefix of the tile sums times the drift window of the
//                       last walk gives each tile the binades its float sum
//                       can be in; tiles whose entries miss one are listed
//   seqnorm_entries     the listed tiles' entries: a refill (one wave per tile
//                       over the batch's iterates, every listed norm) when a
//                       pair listed more than kSnRefillMin tiles, otherwise the
//                       fix (one block of four waves per listed tile and pair)
//   seqnorm_walk        one block per norm and pair: wave 0 walks the tiles 64
//                       per step (saturating DPP scan of their entries for S's
//                       binade); at a tile whose entry does not apply (a
//                       crossing, a tie, a binade outside its candidates) the
//                       block's other waves make the segment entries of its
//                       remaining segments for binades e, e + 1 on request
//                       (sn_help / sn_helper) and leave the terms in LDS, and
//                       the walker steps the crossing segment term by term
//                       with the reference's two roundings.  It writes the
//                       profile the workspace's next batch predicts from.
//   seqnorm_decide      (HS's pipelined loop) the batch's Logger errors as the
//                       host computes them; the first breaking iteration into
//                       the stop word, after which every kernel of a later
//                       batch returns at once (sn_block_stopped)
// The registration runs the pass on one stream, check and entries on a
// second, the walks on three more (registration.cpp enqueue_norms).
// Predictions only decide how much work the walk and the entries do: the
// walk's result is the reference's float sum whatever they predicted.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "of2d_device.h"

namespace of2d {
namespace {

constexpr int kSnThreads = 256;                 // table kernels: 4 waves
constexpr int kSnSegs = kSnTile / 64;           // 64-term segments per tile
constexpr int kSnCand = 4;                      // candidate binades per tile and norm
// relative width of the profile's prediction window (tables): a tile takes the
// binades of [P (1 - w), P' / (1 - w)]; the check's tighter window around the
// fp64 prefix lists the tiles it missed for new entries.  0.1 instead of 0.25
// leaves fewer tiles two candidates (the tables pass is fp64-bound): 4096^2
// convergence on 4-5 % faster, profiles/r03_z_seqnorm_window_ab.log
constexpr double kSnWin = 0.1;
constexpr int kSnScan = 1024;                   // seqnorm_check block
constexpr int kSnEmin = -100;  // below 2^-100 the sum is "low": stepped per nonzero term
constexpr int kSnLow = -1000;
constexpr int kSnNonfinite = 1000;
constexpr unsigned kSnSat = 1u << 25;           // saturated sum of m: certainly a crossing
constexpr unsigned kSnLimit = (1u << 24) - 1u;  // largest M + sum that stays in the binade
constexpr unsigned kSnBad = 1u << 31;           // table entry: a tie or NaN among the terms
// header word of a tile / norm
constexpr unsigned kHdrZero = 1u << 30;     // every magnitude of the tile is 0: a no-op
constexpr unsigned kHdrNan = 1u << 29;      // a NaN magnitude
constexpr unsigned kHdrPending = 1u << 28;  // candidates changed: tile entries to recompute
constexpr unsigned kHdrSegReq = 1u << 27;   // segment entries requested (seqnorm_check)
constexpr unsigned kHdrSeg = 1u << 26;      // segment entries valid for the candidates
__host__ __device__ constexpr unsigned hdr_pack(int elo, int nc) {
    return (unsigned)(elo + 512) | ((unsigned)nc << 16);
}
__device__ __forceinline__ int hdr_elo(unsigned h) { return (int)(h & 0xffffu) - 512; }
__device__ __forceinline__ int hdr_nc(unsigned h) { return (int)((h >> 16) & 7u); }

// the wave's lanes where p holds (HIP's __ballot takes an int: a select and a
// compare more per call)
__device__ __forceinline__ unsigned long long sn_ballot(bool p) {
    return __builtin_amdgcn_ballot_w64(p);
}

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
// the float M ulps in binade e, 2^23 <= M <= kSnLimit
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
__device__ __forceinline__ double sn_scale(int e) {
    return __longlong_as_double((long long)(52 - e + 1023) << 52);
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

// A run of terms inside one binade as a function of the parity of M:
// M -> M + (M even ? lo : hi), packed lo | hi << 32.  A term without a tie adds
// m ulps either way; a tie (d rounded to exactly m0 + 1/2 ulps) rounds
// M + m0 + 1/2 to even, i.e. adds m0 or m0 + 1 by the parity of M.  The form is
// closed under composition, so term-level scans compose ties like any other
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

// The increments from an fp32 estimate of the magnitude (round 4).  m(d, e)
// only depends on where t = d 2^(23-e) lies relative to the half-integers
// (the double sum's grid 2^(e-52) moves t by at most 2^-30), and an estimate
// decides it wherever it lies clear of them.  The estimate
//   q = fma(x, x, y*y) (two roundings: rel. error <= 2^-23), v_sqrt_f32 (1 ulp)
// is within 1.5 2^-23 of d relative wherever q is a normal float well inside
// the range (q in [2^-100, 2^120]; exact zeros are exact), so with
// r = rint(t_est): |t_est - r| < 1/2 - (t 2^-19 + 2^-28) (8x the bound) puts
// the exactly rounded t strictly inside (r - 1/2, r + 1/2): m = r < 2^18, no
// tie.  Every other term (near a half-integer, a large term t >= 2^18 whose
// margin is gone, tiny or huge components, NaN) takes the exact fp64 sequence;
// a wave does so only when
// one of its lanes needs it (a fraction of a percent of waves past the first
// tiles), so the pass runs on fp32 arithmetic and one sqrt per term.
struct SnEst {
    float d;   // the estimate of sqrt((double)x^2 + (double)y^2)
    bool ok;   // its error bound holds
    bool nz;   // the magnitude is not exactly 0 (NaN included)
};
__device__ __forceinline__ SnEst sn_est(float x, float y) {
    SnEst v;
    const float q = __builtin_fmaf(x, x, y * y);  // >= 0 (+0 for zeros), or NaN / inf
    v.nz = ((__float_as_uint(x) | __float_as_uint(y)) << 1) != 0u;
    v.d = __builtin_amdgcn_sqrtf(q);  // branch-free: sqrt(0) = 0
    // q in [2^-100, 2^120] on its bit pattern (NaN / inf / tiny fall outside)
    const unsigned qb = __float_as_uint(q) - 0x0D800000u;
    v.ok = qb <= 0x7B800000u - 0x0D800000u || !v.nz;
    return v;
}
// 2^(23-e) as a float (e in [kSnEmin, 127])
__device__ __forceinline__ float sn_scale32(int e) {
    return __uint_as_float((unsigned)(23 - e + 127) << 23);
}
// m of the estimate in the binade of scale32; false where it does not decide
__device__ __forceinline__ bool sn_incr_est(const SnEst &v, float scale32, unsigned &m) {
    const float t = v.d * scale32;
    const float r = rintf(t);
    const float thr = __builtin_fmaf(t, -0x1p-19f, 0.5f - 0x1p-28f);
    m = (unsigned)r;
    return v.ok && fabsf(t - r) < thr;  // never for t >= 2^18 (thr <= 0), inf or NaN
}

// binade of a double bound, clamped to the float range
__device__ __forceinline__ int sn_region_d(double v) {
    if (!(v >= 0x1p-100)) return kSnLow;
    if (v >= 0x1p127) return 127;
    int ex;
    (void)frexp(v, &ex);
    return ex - 1;
}
// candidate binades covering [lo, hi] (at most kSnCand, the top ones kept)
__device__ __forceinline__ unsigned cand_window(double lo, double hi) {
    const int ehi = sn_region_d(hi);
    if (ehi == kSnLow) return hdr_pack(0, 0);
    int elo = sn_region_d(lo);
    if (elo == kSnLow) elo = kSnEmin;
    if (ehi - elo + 1 > kSnCand) elo = ehi - kSnCand + 1;
    return hdr_pack(elo, ehi - elo + 1);
}

template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
    return v;
}

// sum over the wave (values whose total fits 32 bits): DPP inclusive scan,
// the total read from lane 63
__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, true);  // row_bcast:15
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, true);  // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

struct SnWs {
    double *A;              // [nt][2] fp64 tile sums
    unsigned *H;            // [nt][2] headers
    unsigned long long *Z;  // [nt][2] nonzero-segment masks
    unsigned *T;            // [nt][2][kSnCand] tile entries
    unsigned *G;            // [nt][2][kSnCand][kSnSegs] segment entries
    float *prof;            // [2][nt + 1] exact running sum at each tile start; [nt] = total
    double *Pp;             // [2][nt + 1] fp64 prefix at each tile start (seqnorm_check)
    float *tot;             // [2][2] the last two totals per norm (the walk)
    unsigned *list;         // [nt] tiles seqnorm_check listed for seqnorm_fix
    unsigned *cnt;          // [4] list length
    double *tot64;          // [2] fp64 total of this call (seqnorm_total: a slab's offset)
    double *bs;             // [2][nb] block sums, then block offsets (check)
    float *dr;              // [2][nt + 1] the last call's drift at each tile (check, pass 1)
    unsigned *miss;         // [2] raw segments the last walk stepped (its profile's quality)
    unsigned *stamp;        // [1] epoch + iteration + 1 of the call whose check wrote Pp[.][nt]
};
// The profile of the last call that predicts norm n: its own, except for
// |prev| after a call whose prev was zero (the Logger's first update), whose
// |cur - prev| was this |prev|
__device__ __forceinline__ int prof_src(const SnWs &ws, int n) {
    return (n == 1 && ws.tot[2] == 0.0f) ? 0 : n;
}
__device__ __forceinline__ size_t g_index(unsigned b, int n, int c, int s) {
    return (((size_t)b * 2 + n) * kSnCand + c) * kSnSegs + s;
}

// The lane's term of segment `seg` of tile `b`: the vector whose magnitude it
// is (cur - prev, Field::operator- (Field.tpp:305-334), or prev; 0 past the
// grid), loaded ahead of the raw segment that uses it
struct SnSegTerms {
    float2 v;
};
__device__ __forceinline__ SnSegTerms sn_seg_load(const float2 *__restrict__ cur,
                                                  const float2 *__restrict__ prev, int which,
                                                  unsigned b, int seg, unsigned N, int dimx,
                                                  int P) {
    const unsigned L = b * (unsigned)kSnTile + 64u * seg + (threadIdx.x & 63);
    SnSegTerms t{make_float2(0.0f, 0.0f)};
    if (L < N) {
        const unsigned j = L / (unsigned)dimx, i = L - j * (unsigned)dimx;
        const size_t off = (size_t)j * (size_t)P + i;
        const float2 p = prev[off];
        if (which) {
            t.v = p;
        } else {
            const float2 c = cur[off];
            t.v = make_float2(c.x - p.x, c.y - p.y);
        }
    }
    return t;
}

// ---------------------------------------------------------------- tables
// A batch of K consecutive Logger updates of one loop (round 4): pair i reads
// prev = u[i], cur = u[i + 1] and works on workspace ws[i], so the pass over
// K pairs reads K + 1 iterates instead of 2K (the triple kernel's three
// iterates: 4 arrays for 3 updates).  The check, fix and walk take the batch's
// pairs by blockIdx.y / blockIdx.x.
constexpr int kSnMaxJobs = 3;
struct SnJobs {
    const float2 *u[kSnMaxJobs + 1];
    SnWs ws[kSnMaxJobs];
    int use_prof[kSnMaxJobs];
    const double *p_off[kSnMaxJobs];  // check: a row slab's predecessors' fp64 sums
    const float *s_in[kSnMaxJobs];    // walk: a row slab's predecessors' exact sums
    float *out[kSnMaxJobs];
    int *dbg[kSnMaxJobs];
    // a loop's break (the first iteration whose Logger error ends it, see
    // seqnorm_decide): every kernel of a batch whose first iteration t0 lies
    // past it returns at once (its norms are never read)
    const int *stop;
    int t0;
    unsigned tlo, thi;  // the pass: tiles [tlo, thi) (thi 0: all)
    // the pass: pair i's fp64 totals (Pp) and stamps in the 3 groups before
    const double *nq[kSnMaxJobs][3];
    const unsigned *ns[kSnMaxJobs][3];
    unsigned epoch;
};
__device__ __forceinline__ bool sn_stopped(const SnJobs &J) {
    return J.stop &&
           __hip_atomic_load(J.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < J.t0;
}
// The stop word read ONCE per block and shared through LDS: seqnorm_decide
// (another stream) may set it while the block's waves start, and a block
// whose waves decided apart would run its barriers and inter-wave protocols
// (the walk's helper waves) with some waves gone.  Every kernel that tests the
// word calls this first, in all of its threads.
__device__ __forceinline__ bool sn_block_stopped(const SnJobs &J) {
    __shared__ int stopped;
    if (threadIdx.x == 0) stopped = sn_stopped(J) ? 1 : 0;
    __syncthreads();
    return stopped != 0;
}

// segments in flight per wave: a ring of D segment buffers, each reloaded
// with the segment D ahead right after its own is consumed, so a load has
// D - 1 segments' arithmetic to arrive (the pass: 2-4 x (K + 1) float2; the
// fix, one pair: 8 x 2)
// (K = 3: a ring of 2 measured 119 us per three-update pass against 144 for 4,
// whose 155 VGPRs leave 3 waves per SIMD, and 93 for the loads alone;
// profiles/r04g_sn_ring_ab.log)
// the pass's (and refill's) iterate loads non-temporal: its 537 MB per batch
// at 4096^2 would otherwise push the triple's gradient fields out of the MALL
// they stay in between launches (with the exact loop's GI triples, of2d_device.h
// hs3_exact_gradients_from_image: -7 to -10 % per iteration,
// profiles/r05o_gi_nt_ab.log)
#ifndef OF2D_SN_NT
#define OF2D_SN_NT 1
#endif
// the pass scales its profile (the walk of the same pair 12 updates back) by
// the freshest fp64 total of the pair's norms that a later group's check has
// written (3, 6 or 9 updates back; read with relaxed loads, each check stamps
// its totals), extrapolated geometrically, instead of by the trend of the
// profile's own two last totals: 4096^2 texture convergence 128 -> 122 us per
// iteration warm, 148 -> 136 fresh, procedural unchanged
// (profiles/r05t_near_ab.log; an acquire load there cost 30-50 %: each wave
// waits for its L1 invalidate)
#ifndef OF2D_SN_NEAR
#define OF2D_SN_NEAR 1
#endif
#ifndef OF2D_SN_RING3
#define OF2D_SN_RING3 2
#endif
template <int K>
constexpr int sn_ring() { return K == 1 ? 8 : (K == 2 ? 4 : OF2D_SN_RING3); }

// The lane's terms of consecutive segments of one tile: iterates j0 .. j0 + K
// at linear index L = row jj, column ii (the next segment's), 0 past the grid
template <int K>
struct SnLoader {
    unsigned L, ii, jj;
    __device__ __forceinline__ SnLoader(unsigned b, unsigned dimx) {
        L = b * (unsigned)kSnTile + (threadIdx.x & 63);
        jj = L / dimx;
        ii = L - jj * dimx;
    }
    __device__ __forceinline__ void next(const SnJobs &J, int j0, unsigned N, unsigned dimx,
                                         unsigned P, float2 (&v)[K + 1]) {
#pragma unroll
        for (int k = 0; k <= K; k++) v[k] = make_float2(0.0f, 0.0f);
        if (L < N) {
            const size_t off = (size_t)jj * (size_t)P + ii;
#pragma unroll
            for (int k = 0; k <= K; k++) {
#if OF2D_SN_NT
                typedef float v2f __attribute__((ext_vector_type(2)));
                const v2f w = __builtin_nontemporal_load(reinterpret_cast<const v2f *>(J.u[j0 + k] + off));
                v[k] = make_float2(w.x, w.y);
#else
                v[k] = J.u[j0 + k][off];
#endif
            }
        }
        L += 64u;
        ii += 64u;
        while (ii >= dimx) {
            ii -= dimx;
            jj++;
        }
    }
};

// The pass over tile b for pairs 0 .. K - 1 (one wave): per norm the fp64 tile
// sum A (a prediction: fp32 lane sums of the estimates), the nonzero-segment
// mask Z, the header (candidates from the profile, none without one) and, for
// NC candidate binades (0, 1 or 2), the tile entries T.
// Each lane adds its terms' increments (sn_incr_est: fp32 arithmetic, one
// sqrt; the exact fp64 sequence in the waves where a lane's estimate does not
// decide), so a tile entry is one saturating wave sum at the end.  Segment
// entries come from the fix, for the tiles the check lists.
// a header the refill completes: listed by the check (up to kSnCand
// candidates)
__device__ __forceinline__ bool sn_refills(unsigned h) {
    return (h & kHdrPending) && !(h & (kHdrZero | kHdrNan)) && hdr_nc(h) > 0;
}
// RF (sn_refill_tile): hd are the check's headers; only the pending norms with
// at most NC candidates take entries (T and the header, pending cleared), the
// others are left as they are, and A / Z (the pass's) are not written again.
template <int K, int NC, bool RF = false>
__device__ __forceinline__ void sn_wave_pass(const SnJobs &J, unsigned N, int dimx, int P,
                                             unsigned nt, unsigned b, const unsigned (&hd)[K][2]) {
    const int lane = threadIdx.x & 63;
    int nc[K][2];
    float sc32[K][2][kSnCand];
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            nc[i][n] = (!RF || sn_refills(hd[i][n])) ? hdr_nc(hd[i][n]) : 0;
            // a candidate the header does not have gets scale 0: its
            // increments are 0 and decided, so every term computes all of them
            // without a branch
#pragma unroll
            for (int c = 0; c < kSnCand; c++)
                sc32[i][n][c] = c < nc[i][n] ? sn_scale32(hdr_elo(hd[i][n]) + c) : 0.0f;
        }
    constexpr int NCA = NC > 0 ? NC : 1;
    unsigned tl[K][2][NCA];  // the lane's sum of increments per candidate (<= 64 2^25)
    unsigned bl[K][2];       // the lane's tie / NaN candidates (bit c)
    float fs[K][2];
    bool zv[K][2];  // lane s: segment s has a nonzero magnitude
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            fs[i][n] = 0.0f;
            zv[i][n] = false;
            bl[i][n] = 0u;
#pragma unroll
            for (int c = 0; c < NCA; c++) tl[i][n][c] = 0u;
        }
    SnLoader<K> ld(b, (unsigned)dimx);
    constexpr int D = sn_ring<K>();
    float2 cv[D][K + 1];
#pragma unroll
    for (int d = 0; d < D; d++) ld.next(J, 0, N, (unsigned)dimx, (unsigned)P, cv[d]);
    for (int s0 = 0; s0 < kSnSegs; s0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int s = s0 + d;
#pragma unroll
            for (int i = 0; i < K; i++) {
#pragma unroll
                for (int n = 0; n < 2; n++) {
                    // Field::operator- (Field.tpp:305-334) for |cur - prev|
                    const float x = n ? cv[d][i].x : cv[d][i + 1].x - cv[d][i].x;
                    const float y = n ? cv[d][i].y : cv[d][i + 1].y - cv[d][i].y;
                    const SnEst v = sn_est(x, y);
                    const bool nz = sn_ballot(v.nz) != 0ull;
                    zv[i][n] = lane == s ? nz : zv[i][n];
                    unsigned m[NCA];
                    bool unc = !v.ok;
#pragma unroll
                    for (int c = 0; c < NCA; c++) {
                        m[c] = 0u;
                        if (NC > 0) unc |= !sn_incr_est(v, sc32[i][n][c], m[c]);
                    }
                    float dv = v.d;
                    if (sn_ballot(unc)) {
                        // tiny / huge / non-finite components or an undecided
                        // increment: the exact fp64 magnitude and sequence (the
                        // same m where the estimate decided).  The empty asm
                        // keeps the fp64 work inside this rare branch.
                        float xx = x, yy = y;
                        asm volatile("" : "+v"(xx), "+v"(yy));
                        const double dd = sn_mag(xx, yy);
                        dv = v.ok ? dv : (float)dd;
                        const int e0 = hdr_elo(hd[i][n]);
                        if (NC > 0)
#pragma unroll
                            for (int c = 0; c < NCA; c++) {
                                bool bad = false;
                                const double sc = c < nc[i][n] ? sn_scale(e0 + c) : 0.0;
                                m[c] = sn_incr(dd, sc, bad);
                                bl[i][n] |= bad ? 1u << c : 0u;
                            }
                    }
                    fs[i][n] += dv;  // a prediction only (the check's prefix)
                    if (NC > 0)
#pragma unroll
                        for (int c = 0; c < NCA; c++) tl[i][n][c] += m[c];
                }
            }
            if (s0 + D < kSnSegs) ld.next(J, 0, N, (unsigned)dimx, (unsigned)P, cv[d]);
        }
    }
    auto sat = [](unsigned p, unsigned x) {
        return ((p | x) & kSnBad) | sn_sat(p & ~kSnBad, x & ~kSnBad);
    };
#pragma unroll
    for (int i = 0; i < K; i++) {
        const SnWs &ws = J.ws[i];
#pragma unroll
        for (int n = 0; n < 2; n++) {
            if (RF && !sn_refills(hd[i][n])) continue;
            unsigned hh = RF ? (hd[i][n] & ~kHdrPending) : hd[i][n];
            if (NC > 0) {
                unsigned tv = 0u;
                bool anybad = false;
#pragma unroll
                for (int c = 0; c < NCA; c++) {
                    if (c >= nc[i][n]) continue;
                    const bool bad = sn_ballot((bl[i][n] >> c) & 1u) != 0ull;
                    const unsigned l = tl[i][n][c];
                    const unsigned t =
                        wave_reduce((l < kSnSat ? l : kSnSat), sat) | (bad ? kSnBad : 0u);
                    if (lane == c) tv = t;
                    anybad |= bad;
                }
                if (lane < nc[i][n]) ws.T[(2 * (size_t)b + n) * kSnCand + lane] = tv;
                (void)anybad;  // a tie or NaN: the entry fails in the walk, which resolves it
            }
            if (RF) {
                if (lane == 0) ws.H[2 * (size_t)b + n] = hh;
                continue;
            }
            const double a = wave_reduce((double)fs[i][n], [](double p, double x) { return p + x; });
            const unsigned long long zm = sn_ballot(zv[i][n]);
            if (zm == 0ull) hh = kHdrZero;  // every magnitude exactly 0
            else if (a != a) hh = hdr_pack(0, 0) | kHdrNan;
            if (lane == 0) {
                ws.A[2 * (size_t)b + n] = a;
                ws.Z[2 * (size_t)b + n] = zm;
                ws.H[2 * (size_t)b + n] = hh;
            }
        }
    }
}

// The fix's tile entries of one listed tile b of pair j, by the block's four
// waves (16 consecutive segments each): for each norm whose header is pending
// (the check's new candidates, up to four), each lane adds its terms'
// increments as the pass does; the waves' saturating sums meet in LDS.  The
// walk makes any segment entries it needs itself, so the fix makes none.
__device__ void sn_block_fix(const SnJobs &J, int j, unsigned N, int dimx, int P, unsigned b) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    const SnWs &ws = J.ws[j];
    constexpr int kW = kSnThreads / 64, kSegs = kSnSegs / kW;
    unsigned hd[2];
    int nc[2];
    float sc[2][kSnCand];
#pragma unroll
    for (int n = 0; n < 2; n++) {
        hd[n] = (unsigned)__builtin_amdgcn_readfirstlane((int)ws.H[2 * (size_t)b + n]);
        nc[n] = (hd[n] & kHdrPending) ? hdr_nc(hd[n]) : 0;
#pragma unroll
        for (int c = 0; c < kSnCand; c++)
            sc[n][c] = c < nc[n] ? sn_scale32(hdr_elo(hd[n]) + c) : 0.0f;
    }
    unsigned tl[2][kSnCand] = {}, bl[2] = {0u, 0u};
    SnSegTerms tv[kSegs][2];
#pragma unroll
    for (int k = 0; k < kSegs; k++)
#pragma unroll
        for (int n = 0; n < 2; n++)
            tv[k][n] = nc[n] ? sn_seg_load(J.u[j + 1], J.u[j], n, b, w * kSegs + k, N, dimx, P)
                             : SnSegTerms{make_float2(0.0f, 0.0f)};
#pragma unroll
    for (int k = 0; k < kSegs; k++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            if (!nc[n]) continue;
            const float x = tv[k][n].v.x, y = tv[k][n].v.y;
            const SnEst v = sn_est(x, y);
            unsigned m[kSnCand];
            bool unc = !v.ok;
#pragma unroll
            for (int c = 0; c < kSnCand; c++) unc |= !sn_incr_est(v, sc[n][c], m[c]);
            if (sn_ballot(unc)) {
                const double dd = sn_mag(x, y);
#pragma unroll
                for (int c = 0; c < kSnCand; c++) {
                    bool bad = false;
                    m[c] = sn_incr(dd, c < nc[n] ? sn_scale(hdr_elo(hd[n]) + c) : 0.0, bad);
                    bl[n] |= bad ? 1u << c : 0u;
                }
            }
#pragma unroll
            for (int c = 0; c < kSnCand; c++) tl[n][c] += m[c];
        }
    auto sat = [](unsigned p, unsigned x) {
        return ((p | x) & kSnBad) | sn_sat(p & ~kSnBad, x & ~kSnBad);
    };
    __shared__ unsigned part[kW][2][kSnCand];
#pragma unroll
    for (int n = 0; n < 2; n++)
#pragma unroll
        for (int c = 0; c < kSnCand; c++) {
            if (c >= nc[n]) continue;
            const bool bad = sn_ballot((bl[n] >> c) & 1u) != 0ull;
            const unsigned l = tl[n][c];
            const unsigned t = wave_reduce(l < kSnSat ? l : kSnSat, sat) | (bad ? kSnBad : 0u);
            if (lane == 0) part[w][n][c] = t;
        }
    __syncthreads();
    if (w == 0) {
#pragma unroll
        for (int n = 0; n < 2; n++) {
            if (!nc[n]) continue;
            if (lane < nc[n]) {
                unsigned t = part[0][n][lane];
                for (int q = 1; q < kW; q++) t = sat(t, part[q][n][lane]);
                ws.T[(2 * (size_t)b + n) * kSnCand + lane] = t;
            }
            if (lane == 0) ws.H[2 * (size_t)b + n] = hd[n] & ~(kHdrPending | kHdrSegReq);
        }
    }
    __syncthreads();  // part is reused by the block's next tile
}

// the pass over every tile: one wave per tile, K pairs; the candidate count
// picks the form (none: no profile; one or two: the usual); tiles where the
// profile's window spans more binades (the first ones) are left to the fix
#ifndef OF2D_SN_WPE
#define OF2D_SN_WPE 1
#endif
template <int K>
__global__ __launch_bounds__(kSnThreads) __attribute__((amdgpu_waves_per_eu(OF2D_SN_WPE)))
void seqnorm_tables(unsigned N, int dimx, int P, unsigned nt, SnJobs J) {
    if (sn_block_stopped(J)) return;
    if (blockIdx.x == 0 && threadIdx.x < 4 && J.tlo == 0)
#pragma unroll
        for (int i = 0; i < K; i++) J.ws[i].cnt[threadIdx.x] = 0;  // seqnorm_check's list
    const unsigned b = J.tlo + (unsigned)__builtin_amdgcn_readfirstlane(
                                   (int)(blockIdx.x * (kSnThreads / 64) + threadIdx.x / 64));
    if (b >= (J.thi ? J.thi : nt)) return;
    unsigned hd[K][2];
    int ncmax = 0;
#pragma unroll
    for (int i = 0; i < K; i++) {
        const SnWs &ws = J.ws[i];
#pragma unroll
        for (int n = 0; n < 2; n++) {
            unsigned h = hdr_pack(0, 0);
            if (J.use_prof[i]) {
                // the last call's running sums scaled by the trend of its
                // totals (|cur - prev| shrinks from update to update)
                const int src = prof_src(ws, n);
                const float *pr = ws.prof + (size_t)src * (nt + 1);
                const float t0 = ws.tot[2 * src], t1 = ws.tot[2 * src + 1];
                double r = (src == n && t1 > 0.0f && t0 > 0.0f) ? (double)t0 / t1 : 1.0;
                r = r < 0.25 ? 0.25 : (r > 4.0 ? 4.0 : r);
#if OF2D_SN_NEAR
                if (src == n) {
                    const double q12 = ws.Pp[(size_t)n * (nt + 1) + nt];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const double *qp = J.nq[i][k];
                        if (!qp || !(q12 > 0.0) || J.t0 + i < 3 * (k + 1)) break;
                        const unsigned want = J.epoch + (unsigned)(J.t0 + i - 3 * (k + 1)) + 1u;
                        // relaxed device-scope loads (no acquire: its cache
                        // invalidation would cost every wave beside this one);
                        // a total older than its stamp only predicts worse
                        if (__hip_atomic_load(J.ns[i][k], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) != want)
                            continue;
                        const double qk = __longlong_as_double(__hip_atomic_load(
                            reinterpret_cast<const long long *>(qp + (size_t)n * (nt + 1) + nt),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        if (qk > 0.0 && qk < INFINITY) {
                            // Q(t) = Qk (Qk / Q12)^(d / (12 - d)), d = 3 (k + 1)
                            const float e = 12.0f / (float)(12 - 3 * (k + 1));
                            const float lr = __builtin_amdgcn_logf((float)(qk / q12));
                            float rf = __builtin_amdgcn_exp2f(e * lr);
                            rf = rf < 0.0625f ? 0.0625f : (rf > 16.0f ? 16.0f : rf);
                            r = rf;
                        }
                        break;
                    }
                }
#endif
                h = cand_window((double)pr[b] * r * (1.0 - kSnWin),
                                (double)pr[b + 1] * r / (1.0 - kSnWin));
            }
            hd[i][n] = (unsigned)__builtin_amdgcn_readfirstlane((int)h);  // uniform
            ncmax = max(ncmax, hdr_nc(hd[i][n]));
        }
    }
    if (ncmax > 2) {
        // more candidates than the pass's fixed form: the fix makes this
        // tile's entries (rare: tiles where the sum still climbs binades)
#pragma unroll
        for (int i = 0; i < K; i++)
#pragma unroll
            for (int n = 0; n < 2; n++)
                if (hdr_nc(hd[i][n])) hd[i][n] |= kHdrPending;
        ncmax = 0;
    }
    if (ncmax == 0) sn_wave_pass<K, 0>(J, N, dimx, P, nt, b, hd);
    else if (ncmax == 1) sn_wave_pass<K, 1>(J, N, dimx, P, nt, b, hd);
    else sn_wave_pass<K, 2>(J, N, dimx, P, nt, b, hd);
}

// The check's listed tiles, when there are many (a loop's first batches,
// which have no profile, or a misprediction): one wave per tile reads the
// batch's K + 1 iterates once and makes the entries of every pending norm,
// as the pass does — 4 arrays per tile against the fix's 2 per listed pair,
// and the pass's lane-sum form (seqnorm_entries, when a pair of the batch
// listed more than kSnRefillMin tiles).
#ifndef OF2D_SN_REFILL_MIN
#define OF2D_SN_REFILL_MIN 512  // A/B build knob
#endif
constexpr unsigned kSnRefillMin = OF2D_SN_REFILL_MIN;
template <int K>
__device__ __forceinline__ void sn_refill_tile(const SnJobs &J, unsigned N, int dimx, int P,
                                               unsigned nt, unsigned b) {
    unsigned hd[K][2];
    int ncmax = 0;
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
        for (int n = 0; n < 2; n++) {
            hd[i][n] = (unsigned)__builtin_amdgcn_readfirstlane((int)J.ws[i].H[2 * (size_t)b + n]);
            if (sn_refills(hd[i][n])) ncmax = max(ncmax, hdr_nc(hd[i][n]));
        }
    // two candidates (the usual window), or up to four (the prefix's wide
    // window of a loop's first batches)
    if (ncmax > 2) sn_wave_pass<K, kSnCand, true>(J, N, dimx, P, nt, b, hd);
    else if (ncmax > 0) sn_wave_pass<K, 2, true>(J, N, dimx, P, nt, b, hd);
}

// fp64 prefix of the tile sums (a prediction: any order) -> the binades the
// float sum can be in across each tile: the prefix times the last call's
// drift of the float sum from it (use_prof; 1/64 either side), or the prefix
// alone (1/16 either side).  A tile whose entries miss one is listed for new
// tile entries (pending); the walk makes the segment entries of the tiles it
// resolves itself (sn_help).  Three launches over
// every tile: (1) the last call's drift at each tile (read before this call
// rewrites Pp) and the sums of blocks of kSnChk tiles, (2) one block scans the
// block sums, (3) each block scans its tiles from its offset and checks them.
// (A single 1024-thread block over every tile took 22 us at 4096^2 and 120
// us at 8192^2, 600 us when it waited for CUs behind a triple launch.)
constexpr int kSnChk = 256;  // tiles per block of the check
// (A gate that skipped the check while the last walk on the workspace had
// resolved few tiles was tried in round 4: one overshooting trend scaling of
// a profile then cost a walk thousands of resolves; the check's drift-
// corrected fp64 prefix predicts well, so it runs for every call.)
// without a usable profile (a loop's first four groups) the float sum is taken
// to lie in [P lo, P' 17/16] of the fp64 prefix P: lo = 1/2 (two candidates,
// mostly) instead of 1/16 (four) leaves the refill half the increments; the
// 4096^2 loops' float sums stay within 5 % of P (a grid whose sum drifts
// further only costs the walk term-level steps in those groups): fresh texture
// 136-137 -> 131-132 us per iteration (profiles/r05aa_wide_lo_ab.log)
#ifndef OF2D_SN_WIDE_LO
#define OF2D_SN_WIDE_LO 0.5
#endif
constexpr double kSnWideLo = OF2D_SN_WIDE_LO;
constexpr unsigned kSnMissMax = 256;  // raw segments of a walk whose profile still predicts
__device__ __forceinline__ double sn_drift(const SnWs &ws, unsigned nt, int src, unsigned b) {
    const double f = ws.prof[(size_t)src * (nt + 1) + b], q = ws.Pp[(size_t)src * (nt + 1) + b];
    return (q > 0.0 && f > 0.0 && f < INFINITY) ? f / q : 1.0;
}
__global__ __launch_bounds__(kSnChk) void seqnorm_check_sums(unsigned nt, SnJobs J) {
    if (sn_block_stopped(J)) return;
    const SnWs &ws = J.ws[blockIdx.y];
    const int use_prof = J.use_prof[blockIdx.y];
    const unsigned b = blockIdx.x * kSnChk + threadIdx.x;
    __shared__ double sh[2][kSnChk / 64];
    for (int n = 0; n < 2; n++) {
        if (b <= nt)
            ws.dr[(size_t)n * (nt + 1) + b] =
                use_prof ? (float)sn_drift(ws, nt, prof_src(ws, n), b) : 1.0f;
        const double t = wave_reduce(b < nt ? ws.A[2 * (size_t)b + n] : 0.0,
                                     [](double p, double x) { return p + x; });
        if ((threadIdx.x & 63) == 0) sh[n][threadIdx.x / 64] = t;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        double t = 0.0;
        for (int k = 0; k < kSnChk / 64; k++) t += sh[threadIdx.x][k];
        ws.bs[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = t;
    }
}
// exclusive scan of the nb block sums (in place) plus p_off (a row slab's
// predecessors: the prediction is of the global running sum); Pp[nt] <- the
// total
__global__ __launch_bounds__(kSnScan) void seqnorm_check_scan(unsigned nt, unsigned nb, SnJobs J) {
    if (sn_block_stopped(J)) return;
    const SnWs &ws = J.ws[blockIdx.y];
    const double *p_off = J.p_off[blockIdx.y];
    const unsigned chunk = (nb + kSnScan - 1) / kSnScan;
    const unsigned k0 = min(nb, threadIdx.x * chunk), k1 = min(nb, k0 + chunk);
    __shared__ double sh[2][kSnScan];
    for (int n = 0; n < 2; n++) {
        double t = 0.0;
        for (unsigned k = k0; k < k1; k++) t += ws.bs[(size_t)n * nb + k];
        sh[n][threadIdx.x] = t;
    }
    __syncthreads();
    for (int o = 1; o < kSnScan; o <<= 1) {
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
    double total[2];
    for (int n = 0; n < 2; n++) {
        double run = (threadIdx.x ? sh[n][threadIdx.x - 1] : 0.0) + (p_off ? p_off[n] : 0.0);
        for (unsigned k = k0; k < k1; k++) {
            const double t = ws.bs[(size_t)n * nb + k];
            ws.bs[(size_t)n * nb + k] = run;
            run += t;
        }
        total[n] = run;
    }
    if (threadIdx.x == kSnScan - 1) {
        // the profile predicts the drift of the float sum from the fp64 one
        // only while the sums stay alike: the drift comes mostly from terms
        // that vanish below half an ulp of the running sum, which moves with
        // the terms' size (ws.cnt[1 + n]: the profile of norm n is usable)
        // and while they predicted it: a walk that stepped many raw segments
        // (binades its tiles' candidates missed) leaves a profile whose drift
        // has moved on, and the next call on the workspace takes the wide window
        // (2: totals within 1.25x, the drift +-1/64; 1: within 2.5x, +-1/32;
        // 3: further apart, +-1/16 — the drift moves far less than the sums:
        // early in the 4096^2 texture loop the totals of a workspace's calls
        // twelve updates apart differ 2-5x, its drift by <= 5 %; 0: no usable
        // profile, the prefix alone)
        for (int n = 0; n < 2; n++) {
            const int src = prof_src(ws, n);
            const double old = ws.Pp[(size_t)src * (nt + 1) + nt];
            const double q = old > 0.0 ? total[n] / old : 0.0;
            const bool ok = total[n] > 0.0 && ws.miss[src] <= kSnMissMax;
            ws.cnt[1 + n] = !ok ? 0u : (q < 1.25 && q > 0.8) ? 2u : (q < 2.5 && q > 0.4) ? 1u : 3u;
        }
        for (int n = 0; n < 2; n++) ws.Pp[(size_t)n * (nt + 1) + nt] = total[n];
        // the totals' iteration for a later group's pass (OF2D_SN_NEAR)
        __hip_atomic_store(ws.stamp, J.epoch + (unsigned)(J.t0 + (int)blockIdx.y) + 1u,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ __launch_bounds__(kSnChk) void seqnorm_check(unsigned nt, SnJobs J) {
    if (sn_block_stopped(J)) return;
    const SnWs &ws = J.ws[blockIdx.y];
    const int use_prof = J.use_prof[blockIdx.y];
    const unsigned b = blockIdx.x * kSnChk + threadIdx.x;
    const bool active = b < nt;
    const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
    double a[2], Pb[2];
    unsigned h[2];
    float d0[2], d1[2];
    __shared__ double sw[2][kSnChk / 64];
    for (int n = 0; n < 2; n++) {
        a[n] = active ? ws.A[2 * (size_t)b + n] : 0.0;
        h[n] = active ? ws.H[2 * (size_t)b + n] : 0u;
        d0[n] = active ? ws.dr[(size_t)n * (nt + 1) + b] : 1.0f;
        d1[n] = active ? ws.dr[(size_t)n * (nt + 1) + b + 1] : 1.0f;
        // the block's exclusive prefix: a wave scan, then the waves before
        double x = a[n];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) sw[n][w] = x;
        Pb[n] = x - a[n];
    }
    __syncthreads();
    for (int n = 0; n < 2; n++) {
        double off = ws.bs[(size_t)n * gridDim.x + blockIdx.x];
        for (int k = 0; k < w; k++) off += sw[n][k];
        Pb[n] += off;
    }
    if (!active) return;
    // the window's low end without a profile: kSnWideLo up to 2^25 terms, then
    // scaled down with the count to the 1/16 floor (past 2^24 terms the float
    // sum stagnates further behind the prefix as the grid grows: 8192^2 1/4,
    // 16384^2 1/16) — a prediction only, the walk is exact either way
    const double wide_lo = fmax(1.0 / 16, kSnWideLo * fmin(1.0, 8192.0 / (double)nt));
    bool listed = false;
    for (int n = 0; n < 2; n++) {
        if (!(h[n] & (kHdrZero | kHdrNan)) && a[n] < INFINITY && Pb[n] < INFINITY) {
            // with a usable profile: the prefix times its drift, 1/64 either
            // side; without: the float sum below the fp64 prefix by up to a
            // factor 16 (the kSnCand binades below 1/16 above it: past 2^24
            // terms most small terms vanish below half an ulp and the float
            // sum falls well behind; a miss costs the walk term-level steps)
            const unsigned pq = use_prof ? ws.cnt[1 + n] : 0u;
            const double wd = pq == 2 ? 1.0 / 64 : (pq == 1 ? 1.0 / 32 : 1.0 / 16);
            const unsigned want =
                pq ? cand_window(Pb[n] * d0[n] * (1.0 - wd), (Pb[n] + a[n]) * d1[n] * (1.0 + wd))
                   : cand_window(Pb[n] * wide_lo, (Pb[n] + a[n]) * (1.0 + 1.0 / 16));
            const int wl = hdr_elo(want), wn = hdr_nc(want), hl = hdr_elo(h[n]), hn = hdr_nc(h[n]);
            unsigned hh = h[n];
            // (a header the pass left pending, its window wider than two
            // candidates, takes the check's narrower one)
            if (wn > 0 && ((h[n] & kHdrPending) || wl < hl || wl + wn > hl + hn))
                hh = want | kHdrPending;
            if (hh != h[n]) ws.H[2 * (size_t)b + n] = hh;
            listed |= (hh & kHdrPending) != 0;
        }
        ws.Pp[(size_t)n * (nt + 1) + b] = Pb[n];
    }
    if (listed) ws.list[atomicAdd(&ws.cnt[0], 1u)] = b;
}

// fp64 total of the tile sums (a slab's contribution to its successors' p_off)
__global__ __launch_bounds__(256) void seqnorm_total(unsigned nt, SnWs ws) {
    double s[2] = {0.0, 0.0};
    for (unsigned b = threadIdx.x; b < nt; b += 256)
        for (int n = 0; n < 2; n++) s[n] += ws.A[2 * (size_t)b + n];
    __shared__ double sh[2][4];
    for (int n = 0; n < 2; n++) {
        const double t = wave_reduce(s[n], [](double a, double x) { return a + x; });
        if ((threadIdx.x & 63) == 0) sh[n][threadIdx.x / 64] = t;
    }
    __syncthreads();
    if (threadIdx.x < 2) ws.tot64[threadIdx.x] = sh[threadIdx.x][0] + sh[threadIdx.x][1] +
                                                  sh[threadIdx.x][2] + sh[threadIdx.x][3];
}

// A row slab's prediction offsets for K pairs, chained in rank order: poff =
// the previous rank's running totals (0 for rank 0), nxt = poff + this slab's
// totals (read by the next rank; only adjacent ranks touch each other's memory)
struct SnTotals {
    const double *p[kSnMaxJobs];
};
__global__ void seqnorm_offset_chain(const double *__restrict__ prev_nxt, SnTotals tot, int K,
                                     double *__restrict__ poff, double *__restrict__ nxt) {
    const int i = threadIdx.x >> 1, n = threadIdx.x & 1;
    if (i < K) {
        const double o = prev_nxt ? prev_nxt[2 * i + n] : 0.0;
        poff[2 * i + n] = o;
        nxt[2 * i + n] = o + tot.p[i][n];
    }
}

// The listed tiles' new entries, one launch: with many listed (a pair of the
// batch over kSnRefillMin) the blocks of row 0 refill every tile, a wave per
// tile; otherwise the fix — pair blockIdx.y's listed tiles, one block per
// tile (sn_block_fix).  (Two launches cost the latency chain check -> walk a
// launch more per batch: 4096^2 procedural 139-142 -> 148-149 us per
// iteration, profiles/r04za_predict_ab.log.)
template <int K>
__global__ __launch_bounds__(kSnThreads) void seqnorm_entries(unsigned N, int dimx, int P,
                                                              unsigned nt, SnJobs J) {
    if (sn_block_stopped(J)) return;
    bool many = false;
#pragma unroll
    for (int i = 0; i < K; i++) many |= J.ws[i].cnt[0] > kSnRefillMin;
    if (many) {
        if (blockIdx.y != 0) return;
        const unsigned w = (unsigned)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
        for (unsigned b = blockIdx.x * (kSnThreads / 64) + w; b < nt;
             b += gridDim.x * (kSnThreads / 64))
            sn_refill_tile<K>(J, N, dimx, P, nt, b);
        return;
    }
    const int j = blockIdx.y;
    const unsigned cnt = J.ws[j].cnt[0];
    for (unsigned k = blockIdx.x; k < cnt; k += gridDim.x) {  // block-uniform
        const unsigned b = (unsigned)__builtin_amdgcn_readfirstlane((int)J.ws[j].list[k]);
        sn_block_fix(J, j, N, dimx, P, b);
    }
}

// ---------------------------------------------------------------- the walk
// Wave scans on DPP (row shifts within rows of 16, then the row broadcasts
// of gfx9): lanes shifted in from outside read 0, the identity of both
// operations.  Earlier lanes come first, so the ordered fn composition holds.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_u(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, true);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ sn_fn dpp_fn(sn_fn v) {
    return fn_make(dpp_u<CTRL, ROWS>(fn_e(v)), dpp_u<CTRL, ROWS>(fn_o(v)));
}
__device__ __forceinline__ unsigned wave_incl_sat(unsigned v) {
    v = sn_sat(dpp_u<0x111, 0xF>(v), v);  // row_shr:1
    v = sn_sat(dpp_u<0x112, 0xF>(v), v);  // row_shr:2
    v = sn_sat(dpp_u<0x114, 0xF>(v), v);  // row_shr:4
    v = sn_sat(dpp_u<0x118, 0xF>(v), v);  // row_shr:8
    v = sn_sat(dpp_u<0x142, 0xA>(v), v);  // row_bcast:15 into rows 1, 3
    v = sn_sat(dpp_u<0x143, 0xC>(v), v);  // row_bcast:31 into rows 2, 3
    return v;
}
__device__ __forceinline__ sn_fn wave_incl_fn(sn_fn v) {
    v = fn_then(dpp_fn<0x111, 0xF>(v), v);
    v = fn_then(dpp_fn<0x112, 0xF>(v), v);
    v = fn_then(dpp_fn<0x114, 0xF>(v), v);
    v = fn_then(dpp_fn<0x118, 0xF>(v), v);
    v = fn_then(dpp_fn<0x142, 0xA>(v), v);
    v = fn_then(dpp_fn<0x143, 0xC>(v), v);
    return v;
}
// the value of the lane below (wave_shr:1), 0 in lane 0
__device__ __forceinline__ unsigned lane_below(unsigned v) { return dpp_u<0x138, 0xF>(v); }
__device__ __forceinline__ sn_fn lane_below(sn_fn v) { return dpp_fn<0x138, 0xF>(v); }
__device__ __forceinline__ unsigned lane_at(unsigned v, int q) {
    return (unsigned)__builtin_amdgcn_readlane((int)v, q);
}
__device__ __forceinline__ int first_lane(unsigned long long m) { return __builtin_ctzll(m); }
__device__ __forceinline__ unsigned long long lanes_from(int k) {
    return k >= 64 ? 0ull : (~0ull << k);
}

// The 64 terms of a segment (lane = term, `tv` its vector) from the exact
// running sum S, term by term where the binade changes.
__device__ float sn_raw_segment(SnSegTerms tv, float S) {
    const int lane = threadIdx.x & 63;
    const double dv = sn_mag(tv.v.x, tv.v.y);
    int pos = 0;
    while (pos < 64) {
        const int e = sn_region(S);
        if (e == kSnNonfinite) {
            // inf stays inf unless a NaN follows; NaN stays NaN
            if (sn_ballot(lane >= pos && dv != dv)) S = __uint_as_float(0x7fc00000u);
            return S;
        }
        const bool low = (e == kSnLow);
        const unsigned M = low ? 0u : sn_mant(S);
        bool bad = false;
        sn_fn f = 0;
        if (lane >= pos) {
            if (low)
                bad = (dv != 0.0);  // NaN too
            else
                f = sn_term_fn(dv, sn_scale(e), bad);
        }
        const sn_fn incl = wave_incl_fn(f);
        const sn_fn excl = lane_below(incl);
        const unsigned R = fn_apply(excl, M);
        const bool fail = lane >= pos && (bad || fn_apply(f, R) > kSnLimit);
        const unsigned long long fm = sn_ballot(fail);
        if (!fm) {
            if (!low) S = sn_make(e, fn_apply(fn_make(lane_at(fn_e(incl), 63), lane_at(fn_o(incl), 63)), M));
            return S;
        }
        const int q = first_lane(fm);
        const float Sq = low ? S : sn_make(e, lane_at(R, q));
        const long long db = __double_as_longlong(dv);
        const double dq = __longlong_as_double(
            (long long)lane_at((unsigned)db, q) | ((long long)lane_at((unsigned)(db >> 32), q) << 32));
        S = (float)((double)Sq + dq);  // Motion.cpp:46
        pos = q + 1;
    }
    return S;
}

// Segment entries made on demand (round 4).  A walk block is the walker wave
// and kSnHelpers helper waves; at a tile whose segment entries the
// workspace lacks for S's binade (a crossing, a tie, a missed prediction) the
// walker posts a request in LDS and the eight waves make the entries of the
// tile's segments from sfrom on for binades e and e + 1 (a crossing goes up
// one binade), segment s by wave s mod 8: ~3 us, against ~18 us for the
// walker alone and ~1.1 us per segment stepped raw.  The check no longer
// lists tiles for segment entries ahead of the walk.
constexpr int kSnHelpers = 7;
constexpr int kSnWalkWaves = 1 + kSnHelpers;
constexpr unsigned kSnHelpExit = 0xffffffffu;
struct SnHelp {
    unsigned seq, done;  // request number (the walker's), helpers finished with it
    unsigned b;
    int e, sfrom;
    unsigned g[2][kSnSegs];  // entries for binades e, e + 1
    float2 v[kSnSegs][64];   // the request's terms (segments >= sfrom; 32 KB)
};

// wave `part`'s share of the request: segments s = sfrom + part + 8k
__device__ void sn_help_part(const float2 *__restrict__ cur, const float2 *__restrict__ prev,
                             int which, unsigned b, int sfrom, int e, unsigned N, int dimx, int P,
                             int part, SnHelp &hp) {
    const int lane = threadIdx.x & 63;
    constexpr int kMax = kSnSegs / kSnWalkWaves;
    SnSegTerms tv[kMax];
#pragma unroll
    for (int k = 0; k < kMax; k++) {
        const int sg = sfrom + part + kSnWalkWaves * k;
        tv[k] = SnSegTerms{make_float2(0.0f, 0.0f)};
        if (sg < kSnSegs) tv[k] = sn_seg_load(cur, prev, which, b, sg, N, dimx, P);
    }
    // the terms stay in LDS for the walker's raw steps in this tile
#pragma unroll
    for (int k = 0; k < kMax; k++) {
        const int sg = sfrom + part + kSnWalkWaves * k;
        if (sg < kSnSegs) hp.v[sg][lane] = tv[k].v;
    }
    const bool top = e >= 127;  // no binade above: its entries force raw steps
    const float sc0 = sn_scale32(e), sc1 = top ? 0.0f : sn_scale32(e + 1);
#pragma unroll
    for (int k = 0; k < kMax; k++) {
        const int sg = sfrom + part + kSnWalkWaves * k;
        if (sg >= kSnSegs) break;
        const float vx = tv[k].v.x, vy = tv[k].v.y;
        const SnEst v = sn_est(vx, vy);
        unsigned m0, m1;
        bool unc = !sn_incr_est(v, sc0, m0);
        unc |= !sn_incr_est(v, sc1, m1);
        bool bad0 = false, bad1 = false;
        if (sn_ballot(unc)) {
            const double dd = sn_mag(vx, vy);
            m0 = sn_incr(dd, sn_scale(e), bad0);
            m1 = top ? 0u : sn_incr(dd, sn_scale(e + 1), bad1);
        }
        const unsigned t0 = wave_sum(m0), t1 = wave_sum(m1);
        const bool b0 = sn_ballot(bad0) != 0ull, b1 = sn_ballot(bad1) != 0ull;
        if (lane == 0) {
            hp.g[0][sg] = (t0 < kSnSat ? t0 : kSnSat) | (b0 ? kSnBad : 0u);
            hp.g[1][sg] = top ? (kSnSat | kSnBad) : (t1 < kSnSat ? t1 : kSnSat) | (b1 ? kSnBad : 0u);
        }
    }
}

// the walker's request: entries of tile b's segments from sfrom for binades
// e and e + 1 into g0, g1 (lane s: segment s)
__device__ void sn_help(SnHelp &hp, unsigned &seq, const float2 *__restrict__ cur,
                        const float2 *__restrict__ prev, int which, unsigned b, int sfrom, int e,
                        unsigned N, int dimx, int P, unsigned &g0, unsigned &g1) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        hp.b = b;
        hp.e = e;
        hp.sfrom = sfrom;
        hp.done = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    seq++;
    if (lane == 0) __hip_atomic_store(&hp.seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    sn_help_part(cur, prev, which, b, sfrom, e, N, dimx, P, 0, hp);
    const long long t0 = wall_clock64();
    bool late = false;
    while (__hip_atomic_load(&hp.done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
           (unsigned)kSnHelpers) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > 100000000ll) {  // 1 s: the helpers are gone, do it alone
            late = true;
            break;
        }
    }
    if (late)
        for (int part = 1; part < kSnWalkWaves; part++)
            sn_help_part(cur, prev, which, b, sfrom, e, N, dimx, P, part, hp);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    g0 = lane >= sfrom ? hp.g[0][lane] : 0u;
    g1 = lane >= sfrom ? hp.g[1][lane] : 0u;
}

// a helper wave: serve the walker's requests until it posts kSnHelpExit
__device__ void sn_helper(SnHelp &hp, const float2 *__restrict__ cur,
                          const float2 *__restrict__ prev, int which, unsigned N, int dimx, int P,
                          int part) {
    const int lane = threadIdx.x & 63;
    unsigned my = 0;
    long long t0 = wall_clock64();
    for (;;) {
        const unsigned sq = __hip_atomic_load(&hp.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (sq == kSnHelpExit) return;
        if (sq == my) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > 3000000000ll) return;  // 30 s idle: the walker is gone
            continue;
        }
        my = sq;
        sn_help_part(cur, prev, which, hp.b, hp.sfrom, hp.e, N, dimx, P, part, hp);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(&hp.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        t0 = wall_clock64();
    }
}

// Tile b from the exact running sum S: its segment entries where one covers
// the binade (the tables' or, where those miss it with more than a few
// segments left, the walk's own), raw segments otherwise (a crossing, a tie,
// the low sum).
__device__ float sn_resolve(const float2 *__restrict__ cur, const float2 *__restrict__ prev,
                            int which, unsigned b, unsigned N, int dimx, int P, float S,
                            unsigned h, const SnWs &ws, int &raw, int &made, SnHelp &hp,
                            unsigned &seq) {
    const int lane = threadIdx.x & 63;
    const int nc = (h & kHdrSeg) ? hdr_nc(h) : 0, elo = hdr_elo(h);
    const unsigned long long zm = ws.Z[2 * (size_t)b + which];
    unsigned g[kSnCand];
#pragma unroll
    for (int c = 0; c < kSnCand; c++) g[c] = c < nc ? ws.G[g_index(b, which, c, lane)] : 0u;
    int s0 = 0;
    int enow = kSnLow;       // gnow0 / gnow1: the made entries of binades enow, enow + 1
    int made_at = -kSnSegs;  // segment at which they were made
    int pf_seg = -1;         // segment whose terms pf holds
    SnSegTerms pf{};
    bool no_more = false;    // made entries served < 4 segments: step raw
    unsigned gnow0 = 0, gnow1 = 0;
    while (s0 < kSnSegs) {
        const int e = sn_region(S);
        const int c = e - elo;
        const bool table = c >= 0 && c < nc;
        const bool valid = e != kSnLow && e != kSnNonfinite;
        const bool mine = enow != kSnLow && (e == enow || e == enow + 1);
        // entries of the binade pair S is in, made by the block's waves (not
        // again in a tile where S left them within 4 segments: a sum still
        // climbing through many binades, e.g. the first tiles; 256^2 config 1)
        if (valid && !table && !mine && enow != kSnLow && s0 - made_at < 4) no_more = true;
        if (valid && !table && !mine && kSnSegs - s0 > 2 && !no_more) {
            sn_help(hp, seq, cur, prev, which, b, s0, e, N, dimx, P, gnow0, gnow1);
            enow = e;
            made_at = s0;
            made++;
        }
        if (valid && (table || e == enow || e == enow + 1)) {
            unsigned gc = table ? g[0] : (e == enow ? gnow0 : gnow1);
#pragma unroll
            for (int k = 1; k < kSnCand; k++)
                if (table && c == k) gc = g[k];
            const unsigned M = sn_mant(S);
            const unsigned v = lane >= s0 ? (gc & ~kSnBad) : 0u;
            const unsigned incl = wave_incl_sat(v);
            const unsigned excl = lane_below(incl);
            const bool fail = lane >= s0 && ((gc & kSnBad) || M + incl > kSnLimit);
            const unsigned long long fm = sn_ballot(fail);
            if (!fm) return sn_make(e, M + lane_at(incl, 63));
            const int q = first_lane(fm);
            S = sn_make(e, M + lane_at(excl, q));  // exact: below the limit
            s0 = q;
        } else if (e == kSnLow) {
            const unsigned long long nz = zm & lanes_from(s0);
            if (!nz) return S;  // every remaining term is 0
            s0 = first_lane(nz);
        }
        // this segment's terms: in LDS from the last request, or loaded
        // (prefetched when the last raw one was s0 - 1, the next one's loads
        // in flight behind its steps)
        SnSegTerms tv;
        if (enow != kSnLow && s0 >= made_at) {
            tv.v = hp.v[s0][lane];
        } else {
            tv = pf_seg == s0 ? pf : sn_seg_load(cur, prev, which, b, s0, N, dimx, P);
            if (s0 + 1 < kSnSegs) {
                pf = sn_seg_load(cur, prev, which, b, s0 + 1, N, dimx, P);
                pf_seg = s0 + 1;
            }
        }
        S = sn_raw_segment(tv, S);
        raw++;
        s0++;
    }
    return S;
}

constexpr int kSnAhead = 8;  // windows loaded per step: the next step's loads hide behind them

// One wave per norm and pair walks the tiles in windows of 64 (lane = tile): the
// saturating scan of the entries for S's binade, a resolve at each tile whose
// entry does not apply.  Writes every tile's start sum into the profile.
// dbg: resolves (per norm), raw segments (per norm), listed tiles, walk and
// resolve clocks, tiles given the walk's own segment entries (per norm).
__global__ __launch_bounds__(64 * kSnWalkWaves) void seqnorm_walk(unsigned N, int dimx, int P,
                                                                   unsigned nt, SnJobs J) {
    if (sn_block_stopped(J)) return;  // one decision for the whole block
    const int job = blockIdx.x >> 1;
    const int n = blockIdx.x & 1;  // 0: |cur - prev|, 1: |prev|
    const int lane = threadIdx.x & 63;
    const float2 *__restrict__ prev = J.u[job];
    const float2 *__restrict__ cur = J.u[job + 1];
    __shared__ SnHelp hp;
    if (threadIdx.x == 0) {
        hp.seq = 0u;
        hp.done = 0u;
    }
    __syncthreads();  // the only barrier: from here wave 0 walks, the others help
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
    if (wv > 0) {
        sn_helper(hp, cur, prev, n, N, dimx, P, wv);
        return;
    }
    unsigned seq = 0;
    const SnWs &ws = J.ws[job];
    const float *__restrict__ s_in = J.s_in[job];
    float *__restrict__ out = J.out[job];
    int *__restrict__ dbg = J.dbg[job];
    float *prof = ws.prof + (size_t)n * (nt + 1);
    __shared__ unsigned lh[kSnAhead][64], lt[kSnAhead][kSnCand][64];
    unsigned hn[kSnAhead], tn[kSnAhead][kSnCand];
    auto load = [&](unsigned b0) {
#pragma unroll
        for (int k = 0; k < kSnAhead; k++) {
            const unsigned t = b0 + 64u * k + lane;
            hn[k] = kHdrZero;
#pragma unroll
            for (int c = 0; c < kSnCand; c++) tn[k][c] = 0;
            if (t < nt) {
                hn[k] = ws.H[2 * (size_t)t + n];
#pragma unroll
                for (int c = 0; c < kSnCand; c++)
                    tn[k][c] = ws.T[(2 * (size_t)t + n) * kSnCand + c];
            }
        }
    };
    // s_in: the exact sum of the terms before this grid (the previous row
    // slab's result), 0 without one
    float S = s_in ? s_in[n] : 0.0f;
    int resolves = 0;
    int raw = 0, made = 0;
    bool nan = false;  // non-finite sum: a NaN magnitude after it
    const long long c0 = wall_clock64();
    long long cres = 0;
    load(0);
    for (unsigned bs = 0; bs < nt; bs += 64u * kSnAhead) {
#pragma unroll
        for (int k = 0; k < kSnAhead; k++) {
            lh[k][lane] = hn[k];
#pragma unroll
            for (int c = 0; c < kSnCand; c++) lt[k][c][lane] = tn[k][c];
        }
        if (bs + 64u * kSnAhead < nt) load(bs + 64u * kSnAhead);
        for (int k = 0; k < kSnAhead && bs + 64u * k < nt; k++) {
            const unsigned b0 = bs + 64u * k, t = b0 + lane;
            const unsigned h = lh[k][lane];
            int start = 0;  // first lane of the window not yet added
            while (start < 64) {
                const int e = sn_region(S);
                if (e == kSnNonfinite) {
                    if (lane >= start && t < nt) prof[t] = S;
                    nan |= sn_ballot(lane >= start && (h & kHdrNan)) != 0ull;
                    break;
                }
                const bool low = (e == kSnLow);
                const unsigned M = low ? 0u : sn_mant(S);
                unsigned v = 0;
                bool fail = false;
                if (lane >= start && !(h & kHdrZero)) {
                    const int c = e - hdr_elo(h);
                    // (pending: the pass left this tile's entries to a fix
                    // that did not run; the resolve takes it)
                    if (low || c < 0 || c >= hdr_nc(h) || (h & kHdrPending)) {
                        fail = true;
                    } else {
                        const unsigned w = lt[k][c][lane];
                        fail = (w & kSnBad) != 0;
                        v = w & ~kSnBad;
                    }
                }
                const unsigned incl = wave_incl_sat(v);
                const unsigned excl = lane_below(incl);
                fail = fail || (lane >= start && M + incl > kSnLimit);
                const unsigned long long fm = sn_ballot(fail);
                const int q = fm ? first_lane(fm) : 64;
                // tile start sums of the lanes up to the first failing one: exact
                if (lane >= start && lane <= q && t < nt)
                    prof[t] = low ? S : sn_make(e, M + excl);
                if (!fm) {
                    if (!low) S = sn_make(e, M + lane_at(incl, 63));
                    break;
                }
                if (!low) S = sn_make(e, M + lane_at(excl, q));
                const long long r0 = wall_clock64();
                S = sn_resolve(cur, prev, n, b0 + q, N, dimx, P, S, lane_at(h, q), ws, raw, made,
                               hp, seq);
                cres += wall_clock64() - r0;
                resolves++;
                start = q + 1;
            }
        }
    }
    if (nan) S = __uint_as_float(0x7fc00000u);
    if (lane == 0) {
        prof[nt] = S;
        ws.tot[2 * n + 1] = ws.tot[2 * n];
        ws.tot[2 * n] = S;
        ws.miss[n] = (unsigned)raw;  // segments its resolves stepped term by term
        out[n] = S;
        if (dbg) {
            dbg[n] = resolves;
            dbg[2 + n] = raw;
            if (n == 0) dbg[4] = (int)ws.cnt[0];
            // wall-clock ticks (100 MHz) of the whole walk and of its resolves
            dbg[5 + n] = (int)(wall_clock64() - c0);
            if (n == 0) dbg[7] = (int)cres;
            dbg[8 + n] = made;
        }
        // the helpers may go
        __hip_atomic_store(&hp.seq, kSnHelpExit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// The loop's break on the device: the Logger error of each pair of a walked
// batch, as the host's logger_error (registration.cpp; Logger.cpp:37-39 and
// ImageRegistrationOpticalFlow.cpp:131-134: error < 0.001 and iteration > 1),
// the first breaking iteration into *stop (atomicMin, so batches may finish
// in any order), and the sums copied to the host's mapped mirror.
__global__ void seqnorm_decide(const float *__restrict__ seq, int K, int t0, float npx,
                               int *__restrict__ stop, float *__restrict__ host) {
    const int i = threadIdx.x;
    if (i >= K) return;
    const float sd = seq[2 * i], sp = seq[2 * i + 1];
    host[2 * i] = sd;
    host[2 * i + 1] = sp;
    const float prevnorm = sp / npx, diffnorm = sd / npx;
    const float err = prevnorm == 0.0f ? 0.0f : diffnorm / prevnorm;
    if (err < 0.001f && t0 + i > 1) atomicMin(stop, t0 + i);
}

}  // namespace

size_t seqnorm_workspace_bytes(int dimx, int dimy) {
    const size_t N = (size_t)dimx * (size_t)dimy;
    const size_t nt = (N + kSnTile - 1) / kSnTile;
    return nt * (2 * sizeof(double) + 2 * sizeof(unsigned long long) + 2 * sizeof(unsigned) +
                 2 * kSnCand * sizeof(unsigned) + 2 * kSnCand * kSnSegs * sizeof(unsigned) +
                 sizeof(unsigned)) +
           2 * (nt + 1) * (sizeof(double) + sizeof(float)) + 4 * sizeof(float) +
           4 * sizeof(unsigned) + 2 * sizeof(double) +
           2 * ((nt + 1 + kSnChk - 1) / kSnChk) * sizeof(double) + 2 * (nt + 1) * sizeof(float) +
           2 * sizeof(unsigned) + 256;
}

namespace {
SnWs carve(void *ws, unsigned nt) {
    SnWs w;
    w.A = static_cast<double *>(ws);
    w.Z = reinterpret_cast<unsigned long long *>(w.A + 2 * (size_t)nt);
    w.H = reinterpret_cast<unsigned *>(w.Z + 2 * (size_t)nt);
    w.T = w.H + 2 * (size_t)nt;
    w.G = w.T + 2 * (size_t)nt * kSnCand;
    w.Pp = reinterpret_cast<double *>(w.G + 2 * (size_t)nt * kSnCand * kSnSegs);
    w.prof = reinterpret_cast<float *>(w.Pp + 2 * (size_t)(nt + 1));
    w.tot = w.prof + 2 * (size_t)(nt + 1);
    w.list = reinterpret_cast<unsigned *>(w.tot + 4);
    w.cnt = w.list + nt;
    w.tot64 = reinterpret_cast<double *>(
        (reinterpret_cast<uintptr_t>(w.cnt + 4) + 7) & ~static_cast<uintptr_t>(7));
    w.bs = w.tot64 + 2;
    w.dr = reinterpret_cast<float *>(w.bs + 2 * (size_t)((nt + 1 + kSnChk - 1) / kSnChk));
    w.miss = reinterpret_cast<unsigned *>(w.dr + 2 * (size_t)(nt + 1));
    w.stamp = w.miss + 2;  // inside the allocation's slack
    return w;
}
unsigned check_geometry(int dimx, int dimy, int P) {
    const size_t N = (size_t)dimx * (size_t)dimy;
    if (dimx <= 0 || dimy <= 0 || P < dimx || N > 0xffffffffu)
        throw std::invalid_argument("launch_seqnorm: bad geometry");
    return (unsigned)((N + kSnTile - 1) / kSnTile);
}
}  // namespace

namespace {
SnJobs jobs_of(const SeqnormBatch &B, unsigned nt) {
    if (B.K < 1 || B.K > kSnMaxJobs) throw std::invalid_argument("launch_seqnorm: batch size");
    SnJobs J{};
    for (int i = 0; i <= B.K; i++) J.u[i] = B.u[i];
    for (int i = 0; i < B.K; i++) {
        J.ws[i] = carve(B.ws[i], nt);
        J.use_prof[i] = B.use_profile[i] ? 1 : 0;
        J.p_off[i] = B.p_off[i];
        J.s_in[i] = B.s_in[i];
        J.out[i] = B.out[i];
        J.dbg[i] = B.dbg[i];
    }
    J.stop = B.stop;
    J.t0 = B.t0;
    J.tlo = B.tile_lo;
    J.thi = B.tile_hi;
    J.epoch = B.epoch;
    for (int i = 0; i < B.K; i++)
        for (int k = 0; k < 3; k++) {
            J.nq[i][k] = nullptr;
            J.ns[i][k] = nullptr;
            if (B.near[i][k]) {
                const SnWs w = carve(B.near[i][k], nt);
                J.nq[i][k] = w.Pp;
                J.ns[i][k] = w.stamp;
            }
        }
    return J;
}
}  // namespace

void launch_seqnorm_pass(const SeqnormBatch &B, int dimx, int dimy, int P, hipStream_t st) {
    const unsigned nt = check_geometry(dimx, dimy, P);
    const unsigned N = (unsigned)((size_t)dimx * dimy);
    const SnJobs J = jobs_of(B, nt);
    const unsigned hi = B.tile_hi ? std::min(B.tile_hi, nt) : nt;
    if (B.tile_lo >= hi) return;
    const dim3 grid((hi - B.tile_lo + kSnThreads / 64 - 1) / (kSnThreads / 64));
    switch (B.K) {
        case 1: hipLaunchKernelGGL(seqnorm_tables<1>, grid, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
        case 2: hipLaunchKernelGGL(seqnorm_tables<2>, grid, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
        default: hipLaunchKernelGGL(seqnorm_tables<3>, grid, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
    }
    OF2D_HIP(hipGetLastError());
}

void launch_seqnorm_refine(const SeqnormBatch &B, int dimx, int dimy, int P, hipStream_t st) {
    const unsigned nt = check_geometry(dimx, dimy, P);
    const unsigned N = (unsigned)((size_t)dimx * dimy);
    const SnJobs J = jobs_of(B, nt);
    const unsigned nb = (nt + 1 + kSnChk - 1) / kSnChk;  // blocks over tiles 0 .. nt
    hipLaunchKernelGGL(seqnorm_check_sums, dim3(nb, B.K), dim3(kSnChk), 0, st, nt, J);
    hipLaunchKernelGGL(seqnorm_check_scan, dim3(1, B.K), dim3(kSnScan), 0, st, nt, nb, J);
    hipLaunchKernelGGL(seqnorm_check, dim3(nb, B.K), dim3(kSnChk), 0, st, nt, J);
    OF2D_HIP(hipGetLastError());
    // one block per listed tile (up to 1024 per pair at once), or the refill
    const dim3 eg(std::min(nt, 1024u), B.K);
    switch (B.K) {
        case 1: hipLaunchKernelGGL(seqnorm_entries<1>, eg, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
        case 2: hipLaunchKernelGGL(seqnorm_entries<2>, eg, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
        default: hipLaunchKernelGGL(seqnorm_entries<3>, eg, dim3(kSnThreads), 0, st, N, dimx, P, nt, J); break;
    }
    OF2D_HIP(hipGetLastError());
}

void launch_seqnorm_walk(const SeqnormBatch &B, int dimx, int dimy, int P, hipStream_t st) {
    const unsigned nt = check_geometry(dimx, dimy, P);
    const unsigned N = (unsigned)((size_t)dimx * dimy);
    hipLaunchKernelGGL(seqnorm_walk, dim3(2 * B.K), dim3(64 * kSnWalkWaves), 0, st, N, dimx, P, nt,
                       jobs_of(B, nt));
    OF2D_HIP(hipGetLastError());
}

void launch_seqnorm_decide(const float *seq, int K, int t0, double npx, int *stop, float *host,
                           hipStream_t st) {
    if (K < 1 || K > kSnMaxJobs || !seq || !stop || !host)
        throw std::invalid_argument("launch_seqnorm_decide: arguments");
    hipLaunchKernelGGL(seqnorm_decide, dim3(1), dim3(64), 0, st, seq, K, t0, (float)npx, stop,
                       host);
    OF2D_HIP(hipGetLastError());
}

const double *seqnorm_total(int dimx, int dimy, int P, void *ws, hipStream_t st) {
    const unsigned nt = check_geometry(dimx, dimy, P);
    const SnWs w = carve(ws, nt);
    hipLaunchKernelGGL(seqnorm_total, dim3(1), dim3(256), 0, st, nt, w);
    OF2D_HIP(hipGetLastError());
    return w.tot64;
}

void launch_seqnorm_offset_chain(const double *prev_nxt, const double *const *tot, int K,
                                 double *poff, double *nxt, hipStream_t st) {
    if (K < 1 || K > kSnMaxJobs) throw std::invalid_argument("launch_seqnorm_offset_chain: K");
    SnTotals t{};
    for (int i = 0; i < K; i++) t.p[i] = tot[i];
    hipLaunchKernelGGL(seqnorm_offset_chain, dim3(1), dim3(64), 0, st, prev_nxt, t, K, poff, nxt);
    OF2D_HIP(hipGetLastError());
}

void seqnorm_ws_stats(const void *ws, int dimx, int dimy, unsigned *out) {
    const unsigned nt = check_geometry(dimx, dimy, dimx);
    const SnWs w = carve(const_cast<void *>(ws), nt);
    unsigned cnt[4];
    std::vector<unsigned> H(2 * (size_t)nt);
    OF2D_HIP(hipMemcpy(cnt, w.cnt, sizeof cnt, hipMemcpyDeviceToHost));
    OF2D_HIP(hipMemcpy(H.data(), w.H, H.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    for (int k = 0; k < 4; k++) out[k] = cnt[k];
    for (int k = 4; k < 12; k++) out[k] = 0;
    for (size_t b = 0; b < nt; b++)
        for (int n = 0; n < 2; n++) {
            const unsigned h = H[2 * b + n];
            out[4 + n] += (h & kHdrSeg) ? 1u : 0u;
            out[6 + n] += (h & (kHdrZero | kHdrNan)) ? 0u : (unsigned)((h >> 16) & 7u) > 1u;
            out[8 + n] += (h & (kHdrZero | kHdrNan)) ? 0u : (unsigned)((h >> 16) & 7u) == 0u;
        }
}

// single pairs
namespace {
SeqnormBatch one(const float2 *cur, const float2 *prev, void *ws, bool use_profile) {
    SeqnormBatch B;
    B.K = 1;
    B.u[0] = prev;
    B.u[1] = cur;
    B.ws[0] = ws;
    B.use_profile[0] = use_profile;
    return B;
}
}  // namespace

void launch_seqnorm_pass(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                         void *ws, bool use_profile, hipStream_t st) {
    launch_seqnorm_pass(one(cur, prev, ws, use_profile), dimx, dimy, P, st);
}

void launch_seqnorm_refine(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                           void *ws, bool use_profile, const double *p_off, hipStream_t st) {
    SeqnormBatch B = one(cur, prev, ws, use_profile);
    B.p_off[0] = p_off;
    launch_seqnorm_refine(B, dimx, dimy, P, st);
}

void launch_seqnorm_tables(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                           void *ws, bool use_profile, hipStream_t st) {
    const SeqnormBatch B = one(cur, prev, ws, use_profile);
    launch_seqnorm_pass(B, dimx, dimy, P, st);
    launch_seqnorm_refine(B, dimx, dimy, P, st);
}

void launch_seqnorm_walk(const float2 *cur, const float2 *prev, int dimx, int dimy, int P,
                         void *ws, const float *s_in, float *out, int *dbg, hipStream_t st) {
    SeqnormBatch B = one(cur, prev, ws, false);
    B.s_in[0] = s_in;
    B.out[0] = out;
    B.dbg[0] = dbg;
    launch_seqnorm_walk(B, dimx, dimy, P, st);
}

void launch_seqnorm(const float2 *cur, const float2 *prev, int dimx, int dimy, int P, void *ws,
                    bool use_profile, float *out, int *dbg, hipStream_t st) {
    const SeqnormBatch B = one(cur, prev, ws, use_profile);
    launch_seqnorm_pass(B, dimx, dimy, P, st);
    launch_seqnorm_refine(B, dimx, dimy, P, st);
    launch_seqnorm_walk(cur, prev, dimx, dimy, P, ws, nullptr, out, dbg, st);
}

}  // namespace of2d
