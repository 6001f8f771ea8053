// fluid_kernels.hip — viscous-fluid / elastic solver kernels for gfx950.
//
// OpticalFlowFluid::get_update (src/regularization/OpticalFlow/OpticalFlowFluid.cpp:123-140):
//   f = dI * ((It + u.x dI.x) + u.y dI.y)            OpticalFlow.cpp:15-39
//   SOR sweep of the velocity with right-hand side f  OpticalFlowFluid.cpp:7-41
//   R = v - dudx*v.x - dudy*v.y                       :60-90
//   dt = 0.65 / maxabs(R)  (maxabs squares .y twice)  :92-95, Motion.cpp:51-58
//   if dt < 65: u += R*dt                             :97-121, :135-139
// plus the Logger (Logger.cpp:32-51) and the regridding test
// min(det(I + grad u)) < 0.5 (Image.cpp:189-218, ImageRegistrationFluid.cpp:107-124).
//
// The SOR sweep is Gauss-Seidel IN PLACE with i (x) outer and j (y) inner, so
// v(i,j) reads the NEW v at (i-1,j-1), (i-1,j), (i-1,j+1), (i,j-1) and the OLD
// v at (i+1,*), (i,j+1).  Every pixel on the line 2i + j = t depends only on
// smaller t, so the sweep is executed as that wavefront, which reproduces the
// reference's order exactly (bit-identical results):
//   * one wave per strip of 62 interior columns; lane l (1..62) owns column
//     c0 + l and at step s updates row s - 2(l-1) + 1, two rows behind its
//     left neighbour;
//   * the left neighbour's three most recent NEW values and the right
//     neighbour's three upcoming OLD values arrive by cross-lane shuffles —
//     a step costs no LDS and no barrier;
//   * lane 0 is a ghost of the previous strip's last column: it receives those
//     NEW values from the previous strip through 16-byte {x, y, epoch, epoch}
//     granules written and read with single sc1 dwordx4 accesses (a tag-checked
//     hand-off that needs no release/acquire fence, MI355X guide §6 G16 R2),
//     prefetched 8-16 steps ahead; lane 63 is a ghost of the next
//     strip's first column (OLD values, which that strip cannot overwrite
//     before this strip has published the rows that depend on them);
//   * strips are claimed in order through a ticket counter, so a strip only
//     ever waits on a strip that is already running (no deadlock whatever the
//     dispatch order); every spin is bounded and reports through the status
//     word.
#include "of2d_device.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>

namespace of2d {

namespace {
constexpr unsigned kSpinLimit = 1u << 24;

typedef unsigned long long u64;

// rows per block of the element-wise field kernels (64 x 4 threads, 8 rows
// each): few enough partials that the single-block final reductions are short
constexpr int kFieldRows = 32;

struct Grad2 {
    float2 dx, dy;
};
// partial_x / partial_y of the motion on coord2d (gradients.h:9-32): one-sided
// at the borders, (a - b) / 2 inside
__device__ __forceinline__ Grad2 motion_gradients(const float2 *__restrict__ u, long idx, int i,
                                                  int j, int dimx, int dimy, int P) {
    Grad2 d;
    if (i == 0) {
        const float2 a = u[idx + 1], b = u[idx];
        d.dx = make_float2(a.x - b.x, a.y - b.y);
    } else if (i == dimx - 1) {
        const float2 a = u[idx], b = u[idx - 1];
        d.dx = make_float2(a.x - b.x, a.y - b.y);
    } else {
        const float2 a = u[idx + 1], b = u[idx - 1];
        d.dx = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
    }
    if (j == 0) {
        const float2 a = u[idx + P], b = u[idx];
        d.dy = make_float2(a.x - b.x, a.y - b.y);
    } else if (j == dimy - 1) {
        const float2 a = u[idx], b = u[idx - P];
        d.dy = make_float2(a.x - b.x, a.y - b.y);
    } else {
        const float2 a = u[idx + P], b = u[idx - P];
        d.dy = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
    }
    return d;
}

// max / min over a 64 x 4 block (result valid in thread (0,0)); the order of a
// max or min does not change its value
__device__ __forceinline__ float block_max(float m) {
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (m < o) ? o : m;
    }
    __shared__ float red[4];
    if (threadIdx.x == 0) red[threadIdx.y] = m;
    __syncthreads();
    for (int w = 1; w < 4; w++) m = (m < red[w]) ? red[w] : m;
    return m;
}
__device__ __forceinline__ float block_min(float m) {
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (o < m) ? o : m;
    }
    __shared__ float red[4];
    if (threadIdx.x == 0) red[threadIdx.y] = m;
    __syncthreads();
    for (int w = 1; w < 4; w++) m = (red[w] < m) ? red[w] : m;
    return m;
}
// fp64 Logger partials of a 64 x 4 block, fixed order, written by thread (0,0)
__device__ __forceinline__ void block_sum2(double sd, double sp, double *__restrict__ partial) {
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off);
        sp += __shfl_down(sp, off);
    }
    __shared__ double red[2][4];
    if (threadIdx.x == 0) {
        red[0][threadIdx.y] = sd;
        red[1][threadIdx.y] = sp;
    }
    __syncthreads();
    if (threadIdx.x == 0 && threadIdx.y == 0) {
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        partial[2 * blk + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}
// max / min over a 1024-thread block (result valid in thread 0)
__device__ __forceinline__ float wide_max(float m) {
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (m < o) ? o : m;
    }
    __shared__ float red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    for (int w = 1; w < 16; w++) m = (m < red[w]) ? red[w] : m;
    return m;
}
__device__ __forceinline__ float wide_min(float m) {
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (o < m) ? o : m;
    }
    __shared__ float red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    for (int w = 1; w < 16; w++) m = (red[w] < m) ? red[w] : m;
    return m;
}
}  // namespace

// The sweep works on the array vb of the field being relaxed (v) and its
// right-hand side (b), stored SKEWED along the wavefront: pixel (i, j) lives at
// row t = 2i + j, column i, a row being P float2 v then P float2 b (sor_v,
// sor_b).  Every lane of a strip then works on the same row t at each step, so
// a step's loads are two contiguous 512-B row segments (v and b) and its store
// one (row-major storage would make each 64 separate transactions); the
// passes around the sweep that write only b (the force) write whole runs.  Cells of the
// skewed array that are no pixel (j outside [0, dimy)) are padding: a lane
// whose wavefront row lies outside the image reads and writes back its own
// padding cell instead of branching.
//
// Lane l (0..62) owns column c0 + l and at step s works on row s + 1 - 2l;
// lane 63 is a ghost of the next strip's first column (OLD values only).
// Per step and wave:
//   * two DPP wave_shr:1 move the left neighbours' newest outputs one lane to
//     the right; lane 0, which has no left lane, takes the DPP `old` operand,
//     i.e. the ghost column's value (the previous strip's last column, or the
//     image column 0 for strip 0) — the hand-off costs no select;
//   * two DPP wave_shl:1 bring the right neighbour's newest OLD row; older
//     neighbour values slide through registers (L <- LU, R <- RU ...);
//   * the update itself runs on packed fp32 (v_pk_add/v_pk_mul, no
//     contraction: the reference's float operation order, OpticalFlowFluid.cpp:27-35);
//   * one 8-B store of the new value, one 16-B granule store by lane 62; the
//     stores of lanes that own no interior column are dropped by the buffer
//     range check (voffset past num_records), not masked.
// Loads run one group (kSorNB batches of 8 rows) ahead; granules (lane k of a
// vector = ghost row q + k, {x, y, epoch, epoch}) two batches ahead, are
// tag-checked once per batch and rotated one lane per step by DPP.  A granule
// is written by ONE 16-B-aligned dwordx4 sc1 store from one lane and read by
// one 16-B-aligned dwordx4 sc1 load: a single request on both sides, inside
// one 64-B memory sector, so the tag in the upper half vouches for x, y in
// the lower half (the 8-B form, a tag in each half, costs two register moves
// per step: x, y leave the packed result's even register pair; 3.5-5 % per
// sweep, profiles/r02_ab_sor_halftag.log).  Groups whose rows are interior for every lane skip the
// boundary-row select.
namespace {
constexpr int kSorCols = 63;  // real columns per strip (lanes 0..62)
constexpr int kSorB = 8;      // rows per batch
// batches per group: the row loads run one group (kSorNB * 8 rows) ahead.
// 40 rows: 1.4-3.4 % per sweep faster than 32 at 2048^2-8192^2 (the loads
// wait on HBM at 32); 48 rows spilled into AGPR moves with one group per loop
// trip (profiles/r02_x_sor_lead_ab.log), and are 0.3-1.2 % faster than 40 with
// the unrolled interior loop (profiles/r02_ag_sor_lead_unrolled_ab.log)
#ifdef OF2D_SOR_NB  // tools/sor_harness.hip A/B builds
constexpr int kSorNB = OF2D_SOR_NB;
#else
constexpr int kSorNB = 6;
#endif
constexpr int kSorG = kSorB * kSorNB;
#ifdef OF2D_SOR_UNROLL  // tools/sor_harness.hip A/B builds
constexpr int kSorUnroll = OF2D_SOR_UNROLL;
#else
constexpr int kSorUnroll = 3;  // interior groups per loop trip (2: -3 %, 3: -4 %, 4: -4 % per sweep)
#endif
#ifdef OF2D_SOR_GLEAD  // tools/sor_harness.hip A/B builds only
constexpr int kSorGLead = OF2D_SOR_GLEAD;
#else
constexpr int kSorGLead = 2;  // granule vectors are loaded this many batches ahead
#endif
#ifdef OF2D_SOR_GISSUE  // tools/sor_harness.hip A/B builds only
constexpr int kSorGIssue = OF2D_SOR_GISSUE;
#else
constexpr int kSorGIssue = 6;  // ... issued before this step of the batch: a 10-step lead
// (0: 16 steps, 1.4 % slower per sweep; GLEAD 1 with 0: 8 steps, 35 % slower;
// profiles/r02_ah_sor_granule_issue_ab.log)
#endif
#ifdef OF2D_SOR_HTRACE
constexpr int kSorHtMax = 4096;  // batches recorded per strip
#endif
static_assert(kSorGLead >= 1 && kSorGLead <= kSorNB, "granule vectors rotate through GV[kSorNB]");
// cache policy of the row loads / value stores (tools/sor_harness A/B builds
// override them): the row loads are non-temporal (aux 2), 0.5-1 % per sweep
// at 4096^2 and 8192^2 (profiles/r02_w_sor_cache_ab.log)
#ifndef OF2D_SOR_LD_AUX
#define OF2D_SOR_LD_AUX 2
#endif
#ifndef OF2D_SOR_ST_AUX
#define OF2D_SOR_ST_AUX 0
#endif
constexpr unsigned kOob = 0x40000000u;   // voffset beyond num_records: the access is dropped
constexpr int kNumRecords = 0x20000000;  // bytes addressable from a moving rsrc base
constexpr int kRsrcFlags = 0x00020000;

typedef float v2f __attribute__((ext_vector_type(2)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float dpp_shr_old(float old, float x) {  // lane i <- i-1, lane 0 <- old
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), 0x138,
                                                      0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_shl(float x) {  // lane i <- lane i+1 (lane 63 <- 0)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x130, 0xF, 0xF, true));
}
__device__ __forceinline__ v2f lo2(v4u q) { return v2f{__uint_as_float(q.x), __uint_as_float(q.y)}; }
__device__ __forceinline__ v2f hi2(v4u q) { return v2f{__uint_as_float(q.z), __uint_as_float(q.w)}; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, kNumRecords, kRsrcFlags);
}

// lanes 0..7 of a granule vector: tagged with this sweep's epoch, or a ghost
// row outside the image (never published, never used for an interior pixel)
__device__ __forceinline__ bool granules_ready(v4u g, int row0, int dimy, unsigned epoch) {
    const int lane = threadIdx.x;
    const bool ok = lane >= kSorB || (g.z == epoch && g.w == epoch) ||
                    (unsigned)(row0 + lane) >= (unsigned)dimy;
    return __builtin_amdgcn_ballot_w64(ok) == ~0ull;
}

// Slow path of the hand-off: some granule of the batch was not yet published
// when it was prefetched; poll the batch until it is.  Out of line, so the
// fast path's counted vmcnt is not turned into a drain at a loop preheader.
__device__ __attribute__((noinline)) v4u granule_poll(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                                      int soff, int row0, int dimy,
                                                      unsigned epoch, unsigned *status) {
    v4u g = v4u{0u, 0u, 0u, 0u};
    for (unsigned spins = 0; spins < kSpinLimit; spins++) {
        __builtin_amdgcn_s_sleep(1);
        g = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 16 /* sc1 */);
        if (granules_ready(g, row0, dimy, epoch)) return g;
    }
    atomicOr(status, kStatusSpinTimeout);
    return g;
}

template <bool B>
struct Flag {
    static constexpr bool value = B;
};

// ---------------------------------------------------------------- increment
// behind the sweep.  The Fluid sweep's grid carries `nc` more workgroups
// (tickets nstrips .. nstrips + nc - 1, so every strip is running before any
// of them waits) that compute the increment R = v - dudx v.x - dudy v.y and
// the per-tile maxima of increment_kernel (same tiles, same operations, same
// partial slots) on the 64 x 32 tiles whose strips have finished, while later
// strips still relax: the sweep keeps one wave on ~130 of 1024 SIMDs busy, the
// rest of the chip is idle.  Hand-off (MI355X guide G16, the plain-store
// form): each strip stores v as before (plain), and at its end drains
// (s_waitcnt vmcnt(0)), releases (fence release agent: L2 write-back) and one
// lane stores done[strip] = epoch (sc1); a worker polls done[] with sc1 loads,
// then one agent acquire and plain loads.  (sc1 write-through v stores with
// no release: +27 % per 8192^2 sweep, the in-order vmcnt makes the row loads
// wait for stores that now go to HBM; no change at 2048^2, where the array
// sits in the MALL; profiles/r03bc_*.)  Tiles are taken in column-band order from a
// 64-bit counter (each launch adds exactly ntiles + nc, so a launch's grabs
// are that count modulo ntiles + nc); every wait is bounded in time.
struct SorInc {
    const float2 *u;           // the estimate (not written in the launch)
    float2 *R;                 // increment, row-major
    float *part;               // per-tile max of (float)(2 R.y^2), increment_kernel's slots
    unsigned *done;            // per strip: epoch of its last finished sweep
    unsigned long long *ctr;   // [0] role ticket, [1] tile counter
    int nwg, ntiles, nby;      // worker workgroups (4 waves each), tiles, tile rows
};
constexpr unsigned long long kIncWaitTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ unsigned ld_sc1_u32(const unsigned *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one worker wave: tiles until the counter runs out.  Out of line: inlined, its
// registers raised the strips' SGPR spills from 9 to 156 (v_readlane in the
// sweep's loop)
__device__ __attribute__((noinline)) void sor_increment_worker(const float4 *__restrict__ vb, int dimx, int dimy, int P,
                                     int nstrips, unsigned epoch, const SorInc &w,
                                     unsigned *__restrict__ status, bool zu) {
    // the tile's velocities (kSkJ x kSkI, as increment_kernel), one per wave:
    // the waves of a worker workgroup run independent tile loops, so they
    // synchronise only within themselves (LDS ops of one wave run in order)
    __shared__ float2 vts[4][32][64];
    const int lane = threadIdx.x & 63;
    float2 (*vt)[64] = vts[threadIdx.x >> 6];
    const unsigned long long M = (unsigned long long)w.ntiles + 4ull * (unsigned long long)w.nwg;
    const float2 *__restrict__ vb2 = reinterpret_cast<const float2 *>(vb);
    for (;;) {
        int k0 = 0;
        if (lane == 0) k0 = (int)(atomicAdd(&w.ctr[1], 1ull) % M);
        const int k = __builtin_amdgcn_readfirstlane(k0);
        if (k >= w.ntiles) break;
        const int bx = k / w.nby, by = k - bx * w.nby;
        const int i0 = bx * 64, j0 = by * 32;
        // the estimate around the tile (not written in this launch: plain
        // loads), issued before the wait: rows j0-1 .. j0+32 of the lane's
        // column and the side columns of rows j0 .. j0+31, indices clamped
        // into the image (a clamped value is never used, gradients.h's
        // one-sided border taps take the others)
        float2 uc[34], ul[32], ur[32];
        if (zu) {
            // the zero estimate after a regrid: its gradients are +0 exactly as
            // from a zeroed buffer
#pragma unroll
            for (int r = 0; r < 34; r++) {
                uc[r] = make_float2(0.0f, 0.0f);
                if (r >= 1 && r <= 32) ul[r - 1] = ur[r - 1] = uc[r];
            }
        } else {
            const int ic = min(i0 + lane, dimx - 1);
            const int il = max(ic - 1, 0), ir = min(ic + 1, dimx - 1);
#pragma unroll
            for (int r = 0; r < 34; r++) {
                const long row = (long)min(max(j0 - 1 + r, 0), dimy - 1) * P;
                uc[r] = w.u[row + ic];
                if (r >= 1 && r <= 32) {
                    ul[r - 1] = w.u[row + il];
                    ur[r - 1] = w.u[row + ir];
                }
            }
        }
        // strips over the tile's relaxed columns [max(i0, 1), min(i0 + 63, dimx - 2)]
        const int ca = max(i0, 1), cb = min(i0 + 63, dimx - 2);
        if (ca <= cb) {
            const int Ia = (ca - 1) / 63, Ib = min((cb - 1) / 63, nstrips - 1);
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            bool ok = true;
            for (int I = Ib; I >= Ia; I--) {  // the last strip finishes last
                while (ld_sc1_u32(&w.done[I]) != epoch) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > kIncWaitTicks) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(64);
                }
                if (!ok) break;
            }
            if (!ok && lane == 0) atomicOr(status, kStatusSpinTimeout);
        }
        // one agent acquire after the poll (this CU's L1 may hold lines of v
        // from before the strips' release), then plain loads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // v of the tile along its skewed runs (increment_kernel's skew_tile_for_each,
        // the four thread rows in turn)
        {
            const int q = lane >> 4, kk = lane & 15;
            float2 x[4 * 10];
            int slot[4 * 10];
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int it = 0; it < 10; it++) {
                    const int s = 16 * it + 4 * y + q;
                    const int ii = max(0, (s - 30) >> 1) + kk, jj = s - 2 * ii;
                    const bool in = s < 2 * 63 + 32 && ii < 64 && jj >= 0 && jj < 32 &&
                                    i0 + ii < dimx && j0 + jj < dimy;
                    slot[10 * y + it] = in ? jj * 64 + ii : -1;
                    x[10 * y + it] = in ? vb2[sor_v(i0 + ii, j0 + jj, P)] : make_float2(0.0f, 0.0f);
                }
#pragma unroll
            for (int n = 0; n < 40; n++)
                if (slot[n] >= 0) (&vt[0][0])[slot[n]] = x[n];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int i = i0 + lane;
        float m = 0.0f;
#pragma unroll
        for (int rr = 0; rr < 32; rr++) {
            const int j = j0 + rr;
            if (i < dimx && j < dimy) {
                const long idx = (long)j * P + i;
                const float2 v = vt[rr][lane];
                // motion_gradients (gradients.h:9-32) from the rows loaded up front
                const float2 c = uc[rr + 1];
                float2 dx, dy;
                if (i == 0)
                    dx = make_float2(ur[rr].x - c.x, ur[rr].y - c.y);
                else if (i == dimx - 1)
                    dx = make_float2(c.x - ul[rr].x, c.y - ul[rr].y);
                else
                    dx = make_float2((ur[rr].x - ul[rr].x) / 2.0f, (ur[rr].y - ul[rr].y) / 2.0f);
                if (j == 0)
                    dy = make_float2(uc[rr + 2].x - c.x, uc[rr + 2].y - c.y);
                else if (j == dimy - 1)
                    dy = make_float2(c.x - uc[rr].x, c.y - uc[rr].y);
                else
                    dy = make_float2((uc[rr + 2].x - uc[rr].x) / 2.0f,
                                     (uc[rr + 2].y - uc[rr].y) / 2.0f);
                // (v - dudx*v.x) - dudy*v.y (OpticalFlowFluid.cpp:84), as increment_kernel
                const float2 r = make_float2((v.x - dx.x * v.x) - dy.x * v.y,
                                             (v.y - dx.y * v.x) - dy.y * v.y);
                w.R[idx] = r;
                const double yy = (double)r.y;
                const float qq = (float)(yy * yy + yy * yy);
                m = (m < qq) ? qq : m;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float o = __shfl_down(m, off);
            m = (m < o) ? o : m;
        }
        if (lane == 0) w.part[(long)by * ((dimx + 63) / 64) + bx] = m;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // vt is rewritten by the next tile
    }
}
}  // namespace

template <bool kInc>
__global__ __launch_bounds__(kInc ? 256 : 64) void sor_strip_kernel(float4 *__restrict__ vb, int dimx, int dimy,
                                                       int P, float A, float B, float M, float ML,
                                                       v4u *__restrict__ H, long Hstride,
                                                       unsigned epoch,
                                                       unsigned *__restrict__ ticket, int nstrips,
                                                       unsigned *__restrict__ status,
                                                       unsigned long long *__restrict__ trace,
                                                       SorInc inc, FluidCtl ctl) {
    // an iteration past the loop's break: nothing (no ticket taken, so the
    // counters stay a whole number of launches)
    if (fluid_stopped(ctl)) return;
    const int lane = threadIdx.x;
    __shared__ int s_strip;
    if (lane == 0) {
        if constexpr (kInc)
            s_strip = (int)(atomicAdd(&inc.ctr[0], 1ull) %
                            (unsigned long long)(nstrips + inc.nwg));
        else
            s_strip = (int)(atomicAdd(ticket, 1u) % (unsigned)nstrips);
    }
    __syncthreads();
    const int I = __builtin_amdgcn_readfirstlane(s_strip);
    if constexpr (kInc) {
        if (I >= nstrips) {
            sor_increment_worker(vb, dimx, dimy, P, nstrips, epoch, inc, status,
                                 fluid_zero_est(ctl));
            return;
        }
        if (threadIdx.x >= 64) return;  // a strip is one wave; its CU stays to itself
    }
    // optional timeline (tools/sor_harness.hip): start, end, polled batches,
    // shader cycles
    const unsigned long long t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const unsigned long long c_start = trace ? __builtin_amdgcn_s_memtime() : 0;
    unsigned npoll = 0;
    const int c0 = 1 + kSorCols * I;  // lane 0's column
    const int c = c0 + lane;
    const bool active = lane < kSorCols && c <= dimx - 2;
    // vb addressing: at step s every lane is on skewed row 2 c0 + s + 1; a
    // batch rsrc points at (that row for the batch's first step, column c0);
    // a row is P16 bytes, its b half starts P8 bytes in
    const unsigned P16 = (unsigned)P * 16u, P8 = (unsigned)P * 8u;
    const unsigned voff_ld = (unsigned)lane * 8u;  // lanes past dimx read padding cells
    const unsigned voff_st = active ? (unsigned)lane * 8u : kOob;
    const char *vbc0 = reinterpret_cast<const char *>(vb) + (size_t)c0 * 8u;
    // one row of the lane's column: {v.x, v.y, b.x, b.y}
    auto ldrow = [&](__amdgpu_buffer_rsrc_t rs, int soff, auto aux) __attribute__((always_inline)) {
        constexpr int kAux = decltype(aux)::value;
        const v2u v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff_ld, soff, kAux);
        const v2u b = __builtin_amdgcn_raw_buffer_load_b64(rs, voff_ld, soff + (int)P8, kAux);
        return v4u{v.x, v.y, b.x, b.y};
    };
    using Aux0 = std::integral_constant<int, 0>;
    using AuxLd = std::integral_constant<int, OF2D_SOR_LD_AUX>;
    // granules: region I (ghost column of this strip), region I+1 (published)
    const char *gin = reinterpret_cast<const char *>(H + (long)I * Hstride + kSorPadRows);
    const char *gout = reinterpret_cast<const char *>(H + (long)(I + 1) * Hstride + kSorPadRows);
    const unsigned voff_gin = lane < kSorB ? (unsigned)lane * 16u : kOob;
    const unsigned voff_pub = lane == kSorCols - 1 ? 0u : kOob;

    const int s0 = -3;
    const int s1 = dimy + 122;  // lane 62 publishes ghost row dimy - 1 at this step
    // running bases, advanced per batch / group (no 64-bit multiply per
    // batch): vrow = skewed row of the next batch's first step (column c0),
    // prow = the granule row lane 62 publishes at that step, grow = the ghost
    // granule row of the current group's first step + 2
    const char *vrow = vbc0 + (long)(2 * c0 + s0 + 1) * P16;
    const char *prow = gout + (long)(s0 - 123) * 16;
    const char *grow = gin + (long)(s0 + 2) * 16;
    const long vstep = (long)kSorB * P16;

    // window rows r..r+3 of the first step, batches of the first group
    v4u W0, W1, W2, W3, X[kSorNB][kSorB], GV[kSorNB];
    {
        const auto rs = rsrc_at(vrow);
        W0 = ldrow(rs, 0, Aux0{});
        W1 = ldrow(rs, (int)P16, Aux0{});
        W2 = ldrow(rs, 2 * (int)P16, Aux0{});
        W3 = ldrow(rs, 3 * (int)P16, Aux0{});
#pragma unroll
        for (int b = 0; b < kSorNB; b++)
#pragma unroll
            for (int j = 0; j < kSorB; j++) X[b][j] = ldrow(rs, (4 + kSorB * b + j) * (int)P16, Aux0{});
        const auto gr = rsrc_at(grow);
#pragma unroll
        for (int b = 0; b < kSorGLead; b++)
            GV[b] = __builtin_amdgcn_raw_buffer_load_b128(gr, voff_gin, kSorB * b * 16, 16);
    }
    v2f RD = v2f{dpp_shl(__uint_as_float(W1.x)), dpp_shl(__uint_as_float(W1.y))};
    v2f R = v2f{dpp_shl(__uint_as_float(W2.x)), dpp_shl(__uint_as_float(W2.y))};
    v2f RU = v2f{dpp_shl(__uint_as_float(W3.x)), dpp_shl(__uint_as_float(W3.y))};
    v2f LU = v2f{0.0f, 0.0f}, L = LU, D = lo2(W0);
    v2f G = LU;  // lane k: ghost row (step + 2 + k) of the current batch

#define SOR_SHL(x) dpp_shl(x)
#define SOR_SHR(o, x) dpp_shr_old(o, x)
    auto step = [&](auto chk, int s, int j, __amdgpu_buffer_rsrc_t rs,
                    __amdgpu_buffer_rsrc_t ps, v4u xin) {
        const v2f C = lo2(W0), b = hi2(W0), U = lo2(W1);
        // left neighbours' NEW values at rows r+1, r, r-1 (ghost column in lane 0)
        const v2f LD = L;
        L = LU;
        const v2f Gn = v2f{SOR_SHL(G.x), SOR_SHL(G.y)};  // next step's ghost row in lane 0
        LU = v2f{SOR_SHR(G.x, D.x), SOR_SHR(G.y, D.y)};
        G = Gn;
        // OpticalFlowFluid.cpp:27-35, same association, no contraction
        const v2f RL = R + L;
        const v2f s1v = (RL + U) + D;
        const v2f t = ((RU - LU) - RD) + LD;
        const v2f s2v = RL + 0.25f * t.yx;
        const v2f n = A * C + B * ((b - M * s1v) - ML * s2v);
        v2f out = n;
        if constexpr (decltype(chk)::value) {
            const int r = s + 1 - 2 * lane;
            if ((unsigned)(r - 1) >= (unsigned)(dimy - 2)) out = C;  // boundary row: OLD value
        }
        __builtin_amdgcn_raw_buffer_store_b64(
            v2u{__float_as_uint(out.x), __float_as_uint(out.y)}, rs, voff_st, j * (int)P16,
            OF2D_SOR_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(
            v4u{__float_as_uint(out.x), __float_as_uint(out.y), epoch, epoch}, ps,
            voff_pub + (unsigned)j * 16u, 0, 16 /* sc1 */);
        D = out;
        W0 = W1;
        W1 = W2;
        W2 = W3;
        W3 = xin;
        RD = R;
        R = RU;
        RU = v2f{SOR_SHL(__uint_as_float(W3.x)), SOR_SHL(__uint_as_float(W3.y))};
    };
#undef SOR_SHL
#undef SOR_SHR

    auto group = [&](auto chk, int g) {
        const auto gr = rsrc_at(grow);
#pragma unroll
        for (int b = 0; b < kSorNB; b++) {
            const int sb = g + kSorB * b;
            // ghost rows sb+2 .. sb+9: check the tags, start the lead batch's load
            v4u gv = GV[b];
#ifdef OF2D_SOR_HTRACE  // tools/sor_harness.hip: per-batch hand-off timeline
            unsigned long long polled = 0;
#endif
            if (!granules_ready(gv, sb + 2, dimy, epoch)) {
                gv = granule_poll(gr, voff_gin, kSorB * b * 16, sb + 2, dimy, epoch, status);
                npoll++;
#ifdef OF2D_SOR_HTRACE
                polled = 1ull << 63;
#endif
            }
            G = lo2(gv);
#ifdef OF2D_SOR_HTRACE
            if (lane == 0)
                trace[4 * nstrips + (long)I * kSorHtMax + (sb - s0) / kSorB] =
                    __builtin_amdgcn_s_memrealtime() | polled;
#endif
            const auto rs = rsrc_at(vrow);
            const auto ps = rsrc_at(prow);
#pragma unroll
            for (int j = 0; j < kSorB; j++) {
                if (j == kSorGIssue) {  // the lead batch's granules
                    const int bl = b + kSorGLead;  // batch index counted from this group
                    GV[bl % kSorNB] = __builtin_amdgcn_raw_buffer_load_b128(gr, voff_gin,
                                                                            kSorB * bl * 16, 16);
                }
                step(chk, sb + j, j, rs, ps, X[b][j]);
            }
            // batch b of the next group: rows 32 further down
#pragma unroll
            for (int j = 0; j < kSorB; j++) X[b][j] = ldrow(rs, (4 + kSorG + j) * (int)P16, AuxLd{});
            vrow += vstep;
            prow += kSorB * 16;
        }
        grow += kSorG * 16;
    };

    // three loops: head groups with the boundary-row select, interior groups
    // without it, tail groups with it.  The interior loop runs kSorUnroll
    // groups per trip: its back edge copies ~32 row registers (the allocator
    // does not keep the row ring in place across a trip) and waits on their
    // loads, so fewer trips cost less (one group per trip, both kinds of
    // group in one loop: 186 cycles per step of strip 0 at 8192^2; three
    // loops, 3 groups per trip: 164; profiles/r02_af_sor_loops_ab.log)
    int g = s0;
    for (; g <= s1 && g < 124; g += kSorG) group(Flag<true>{}, g);
    for (; g + (kSorUnroll - 1) * kSorG <= s1 && g + kSorUnroll * kSorG - 1 <= dimy - 3;
         g += kSorUnroll * kSorG) {
#pragma unroll
        for (int q = 0; q < kSorUnroll; q++) group(Flag<false>{}, g + q * kSorG);
    }
    for (; g <= s1 && g + kSorG - 1 <= dimy - 3; g += kSorG) group(Flag<false>{}, g);
    for (; g <= s1; g += kSorG) group(Flag<true>{}, g);
    if (trace && lane == 0) {
        trace[4 * I] = t_start;
        trace[4 * I + 1] = __builtin_amdgcn_s_memrealtime();
        trace[4 * I + 2] = npoll;
        trace[4 * I + 3] = __builtin_amdgcn_s_memtime() - c_start;
    }
    if constexpr (kInc) {  // the strip's v stores drained and released, then its flag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
            __hip_atomic_store(&inc.done[I], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int sor_nstrips(int dimx) { return dimx < 3 ? 0 : (dimx - 2 + kSorCols - 1) / kSorCols; }
long sor_granule_stride(int dimy) { return (long)dimy + 2L * kSorPadRows; }
size_t sor_granule_bytes(int dimx, int dimy) {
    return (size_t)(sor_nstrips(dimx) + 1) * (size_t)sor_granule_stride(dimy) * 16u;
}

void launch_sor_traced(float4 *vb, int dimx, int dimy, int P, float mu, float lambda, float omega,
                       void *H, unsigned epoch, unsigned *ticket, unsigned *status,
                       unsigned long long *trace, hipStream_t st, FluidCtl ctl = {}) {
    if (dimx < 3 || dimy < 3) return;  // no interior (OpticalFlowFluid.cpp:23-24)
    const int ns = sor_nstrips(dimx);
    // per-pixel constants of OpticalFlowFluid.cpp:27 evaluated once, same float ops
    const float A = 1.0f - omega;
    const float B = omega / (-6 * mu - 2 * lambda);
    const float ML = mu + lambda;
    hipLaunchKernelGGL(sor_strip_kernel<false>, dim3(ns), dim3(64), 0, st, vb, dimx, dimy, P, A,
                       B, mu, ML, (v4u *)H, sor_granule_stride(dimy), epoch, ticket, ns, status,
                       trace, SorInc{}, ctl);
    OF2D_HIP(hipGetLastError());
}
void launch_sor(float4 *vb, int dimx, int dimy, int P, float mu, float lambda, float omega,
                void *H, unsigned epoch, unsigned *ticket, unsigned *status, hipStream_t st,
                FluidCtl ctl) {
    launch_sor_traced(vb, dimx, dimy, P, mu, lambda, omega, H, epoch, ticket, status, nullptr, st,
                      ctl);
}

// Row-major <-> skewed transfer of a 64 (i) x 32 (j) pixel tile through LDS.
// In the skewed array the tile's pixels lie on local rows s = 2 ii + jj in
// [0, 158), each row a run of at most 16 consecutive columns; a quarter-wave
// (16 lanes) takes one such run, so every skewed access is a contiguous
// 256-B segment (row-major iteration would put each lane of a wave on its own
// skewed row: 64 separate 16-B transactions per wave access).  LDS address
// of (ii, jj) in a [32][64] tile advances by -127 slots per lane along a run:
// 16 lanes on distinct banks.  Block dim3(64, 4).
constexpr int kSkI = 64, kSkJ = 32;
static_assert(kSkJ == kFieldRows && kSkI == 64, "field kernels tile 64 x kFieldRows");
constexpr int kSkIts = 10;  // skewed runs per thread
// pixel (ii, jj) of the thread's run `it`, and whether it is one of the tile's
// pixels inside the image
__device__ __forceinline__ bool skew_slot(int it, int i0, int j0, int dimx, int dimy, int &ii,
                                          int &jj) {
    const int q = threadIdx.x >> 4, k = threadIdx.x & 15;
    const int s = 16 * it + 4 * (int)threadIdx.y + q;  // < 2 * 63 + 31 + 1 = 158
    ii = max(0, (s - 30) >> 1) + k;                    // ceil((s - 31) / 2) + k
    jj = s - 2 * ii;
    return s < 2 * (kSkI - 1) + kSkJ && ii < kSkI && jj >= 0 && jj < kSkJ && i0 + ii < dimx &&
           j0 + jj < dimy;
}
template <class F>
__device__ __forceinline__ void skew_tile_for_each(int i0, int j0, int dimx, int dimy, F f) {
#pragma unroll
    for (int it = 0; it < kSkIts; it++) {
        int ii, jj;
        if (skew_slot(it, i0, j0, dimx, dimy, ii, jj)) f(ii, jj);
    }
}
// vb's b <- f(ii, jj) over the tile's skewed runs (8-B elements, runs of 16
// consecutive columns: whole 128-B segments, no read of v)
template <class F>
__device__ __forceinline__ void skew_tile_set_b(float4 *__restrict__ vb, int i0, int j0, int dimx,
                                                int dimy, int P, F f) {
    float2 *vb2 = reinterpret_cast<float2 *>(vb);
    skew_tile_for_each(i0, j0, dimx, dimy,
                       [&](int ii, int jj) { vb2[sor_b(i0 + ii, j0 + jj, P)] = f(ii, jj); });
}

// vb's b <- force(u, dI, It) (OpticalFlow.cpp:15-39); with pack_v also its v <- v.
// Column 0 (never relaxed) is the ghost column of strip 0: its values go to
// granule region 0 with this sweep's epoch.
__global__ __launch_bounds__(256) void sor_pack_kernel(float4 *__restrict__ vb,
                                                        const float2 *__restrict__ u,
                                                        const float2 *__restrict__ dI,
                                                        const float *__restrict__ It,
                                                        const float2 *__restrict__ v, int dimx,
                                                        int dimy, int P, v4u *__restrict__ H,
                                                        unsigned epoch) {
    __shared__ float4 tile[kSkJ][kSkI];
    const int i0 = blockIdx.x * kSkI, j0 = blockIdx.y * kSkJ;
    const int i = i0 + threadIdx.x;
    for (int r = threadIdx.y; r < kSkJ; r += 4) {
        const int j = j0 + r;
        if (i >= dimx || j >= dimy) break;
        const long idx = (long)j * P + i;
        const float2 m = u[idx], g = dI[idx];
        const float sc = (It[idx] + m.x * g.x) + m.y * g.y;
        float2 x = v ? v[idx] : make_float2(0.0f, 0.0f);
        tile[r][threadIdx.x] = make_float4(x.x, x.y, g.x * sc, g.y * sc);
        if (i == 0 && H) {
            if (!v) x = reinterpret_cast<const float2 *>(vb)[sor_v(0, j, P)];
            H[kSorPadRows + j] = v4u{__float_as_uint(x.x), __float_as_uint(x.y), epoch, epoch};
        }
    }
    __syncthreads();
    if (v) {
        float2 *vb2 = reinterpret_cast<float2 *>(vb);
        skew_tile_for_each(i0, j0, dimx, dimy, [&](int ii, int jj) {
            const float4 q = tile[jj][ii];
            vb2[sor_v(i0 + ii, j0 + jj, P)] = make_float2(q.x, q.y);
            vb2[sor_b(i0 + ii, j0 + jj, P)] = make_float2(q.z, q.w);
        });
    } else {
        skew_tile_set_b(vb, i0, j0, dimx, dimy, P, [&](int ii, int jj) {
            const float4 q = tile[jj][ii];
            return make_float2(q.z, q.w);
        });
    }
}
void launch_sor_pack(float4 *vb, const float2 *u, const float2 *dI, const float *It,
                     const float2 *v, int dimx, int dimy, int P, void *H, unsigned epoch,
                     hipStream_t st) {
    hipLaunchKernelGGL(sor_pack_kernel, dim3((dimx + kSkI - 1) / kSkI, (dimy + kSkJ - 1) / kSkJ),
                       dim3(64, 4), 0, st, vb, u, dI, It, v, dimx, dimy, P, (v4u *)H, epoch);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ regrid pack
// After a fluid regrid (ImageRegistrationFluid.cpp:118-123): set_derivatives
// of the new warped image (IterativeSolver.cpp:22-56, gradients.h:9-32; the
// same taps and operations as gradients_kernel) and the next sweep's force of
// the zeroed estimate into vb's b (get_force with u = +0, the operations of
// sor_pack_kernel), in one pass over a 64 x 32 tile.
__global__ __launch_bounds__(256) void regrid_pack_kernel(
    const float *__restrict__ Iref, const float *__restrict__ Ia, float2 *__restrict__ dI,
    float *__restrict__ It, float4 *__restrict__ vb, int dimx, int dimy, int P,
    v4u *__restrict__ H, unsigned epoch, FluidCtl ctl) {
    // with control words: only after an iteration that regridded
    if (ctl.w && (fluid_stopped(ctl) || !fluid_zero_est(ctl))) return;
    __shared__ float2 fo[kSkJ][kSkI];
    // tiles in a grid-stride loop: a capped grid keeps the launch cheap when
    // the control words make it a no-op (most iterations)
    const int ntx = (dimx + kSkI - 1) / kSkI, ntiles = ntx * ((dimy + kSkJ - 1) / kSkJ);
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int i0 = (tile % ntx) * kSkI, j0 = (tile / ntx) * kSkJ;
    const int i = i0 + threadIdx.x;
    constexpr int NK = kSkJ / 4;
    // taps of every row of the thread first (border rows and columns pick the
    // one-sided taps; rows outside the image read element 0)
    float ia[NK], ib[NK], ja[NK], jb[NK], io[NK], ir[NK];
    bool okk[NK];
    const bool xl = i == 0, xr = !xl && i == dimx - 1;
#pragma unroll
    for (int k = 0; k < NK; k++) {
        const int j = j0 + 4 * k + threadIdx.y;
        okk[k] = i < dimx && j < dimy;
        const unsigned idx = okk[k] ? (unsigned)j * (unsigned)P + (unsigned)i : 0u;
        const bool yl = j == 0, yr = !yl && j == dimy - 1;
        ia[k] = Ia[okk[k] ? (xr ? idx : idx + 1) : 0];
        ib[k] = Ia[okk[k] ? (xl ? idx : idx - 1) : 0];
        ja[k] = Ia[okk[k] ? (yr ? idx : idx + P) : 0];
        jb[k] = Ia[okk[k] ? (yl ? idx : idx - P) : 0];
        io[k] = Ia[idx];
        ir[k] = Iref[idx];
    }
#pragma unroll
    for (int k = 0; k < NK; k++) {
        if (!okk[k]) continue;
        const int rr = 4 * k + threadIdx.y;
        const int j = j0 + rr;
        const long idx = (long)j * P + i;
        const bool yl = j == 0, yr = !yl && j == dimy - 1;
        const float gx = (xl || xr) ? ia[k] - ib[k] : (ia[k] - ib[k]) / 2.0f;
        const float gy = (yl || yr) ? ja[k] - jb[k] : (ja[k] - jb[k]) / 2.0f;
        const float t = io[k] - ir[k];
        dI[idx] = make_float2(gx, gy);
        It[idx] = t;
        const float z = 0.0f;  // the estimate after the regrid
        const float sc = (t + z * gx) + z * gy;
        fo[rr][threadIdx.x] = make_float2(gx * sc, gy * sc);
        if (i == 0 && H) {
            const float2 x = reinterpret_cast<const float2 *>(vb)[sor_v(0, j, P)];
            H[kSorPadRows + j] = v4u{__float_as_uint(x.x), __float_as_uint(x.y), epoch, epoch};
        }
    }
    __syncthreads();
    skew_tile_set_b(vb, i0, j0, dimx, dimy, P, [&](int ii, int jj) { return fo[jj][ii]; });
    __syncthreads();  // fo is rewritten by the block's next tile
    }
}
// blocks of the device-decided regrid pack (a no-op on most iterations: a
// smaller grid is a cheaper no-op, a larger one a faster real pack).  One
// tile per block up to 8192^2: config 4 +0.6-0.7 % against the host-decided
// loop, where 2048 blocks (16 tiles each at 8192^2) made the real packs 38 %
// slower and 8192 blocks gained 0.2 % (profiles/r06f_fluid_packcap_ab.log)
#ifndef OF2D_FLUID_PACK_CAP
#define OF2D_FLUID_PACK_CAP 32768
#endif
void launch_regrid_pack(const float *Iref, const float *Iaux, float2 *dI, float *It, float4 *vb,
                        int dimx, int dimy, int P, void *H, unsigned epoch, hipStream_t st,
                        FluidCtl ctl) {
    const int ntiles = ((dimx + kSkI - 1) / kSkI) * ((dimy + kSkJ - 1) / kSkJ);
    hipLaunchKernelGGL(regrid_pack_kernel, dim3(ctl.w ? std::min(ntiles, OF2D_FLUID_PACK_CAP) : ntiles),
                       dim3(64, 4), 0, st, Iref, Iaux, dI, It, vb, dimx, dimy, P, (v4u *)H,
                       epoch, ctl);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ pointwise force
// OpticalFlow::get_force (OpticalFlow.cpp:15-39): f = dI * ((It + u.x dI.x) + u.y dI.y)
__global__ void force_kernel(const float2 *__restrict__ u, const float2 *__restrict__ dI,
                             const float *__restrict__ It, float2 *__restrict__ f, int dimx,
                             int dimy, int P) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    if (i >= dimx || j >= dimy) return;
    const long idx = (long)j * P + i;
    const float2 m = u[idx], g = dI[idx];
    const float sc = (It[idx] + m.x * g.x) + m.y * g.y;
    f[idx] = make_float2(g.x * sc, g.y * sc);
}
void launch_force(const float2 *u, const float2 *dI, const float *It, float2 *f, int dimx,
                  int dimy, int P, hipStream_t st) {
    hipLaunchKernelGGL(force_kernel, dim3((dimx + 63) / 64, (dimy + 3) / 4), dim3(64, 4), 0, st,
                       u, dI, It, f, dimx, dimy, P);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ increment + maxabs
// R = v - dudx * v.x - dudy * v.y (OpticalFlowFluid.cpp:84), partial_x/y of the
// motion (gradients.h:9-32 on coord2d), and per-block max of (float)(2 y^2)
// (Motion::maxabs, Motion.cpp:51-58)
__global__ __launch_bounds__(256) void increment_kernel(const float2 *__restrict__ u,
                                                        const float4 *__restrict__ vel,
                                                        float2 *__restrict__ R, int dimx, int dimy,
                                                        int P, float *__restrict__ part,
                                                        FluidCtl ctl) {
    if (fluid_stopped(ctl)) return;
    const bool zu = fluid_zero_est(ctl);
    __shared__ float2 vt[kSkJ][kSkI];  // the tile's velocities, read along skewed rows
    const int i0 = blockIdx.x * kSkI, j0 = blockIdx.y * kFieldRows;
    skew_tile_for_each(i0, j0, dimx, dimy, [&](int ii, int jj) {
        vt[jj][ii] = reinterpret_cast<const float2 *>(vel)[sor_v(i0 + ii, j0 + jj, P)];
    });
    __syncthreads();
    const int i = i0 + threadIdx.x;
    float m = 0.0f;
    for (int k = 0; k < kFieldRows / 4; k++) {
        const int j = j0 + 4 * k + threadIdx.y;
        if (i >= dimx || j >= dimy) break;
        const long idx = (long)j * P + i;
        const float2 v = vt[4 * k + threadIdx.y][threadIdx.x];
        // the zero estimate of a regrid: gradients +0, as from a zeroed buffer
        const Grad2 d = zu ? Grad2{make_float2(0.0f, 0.0f), make_float2(0.0f, 0.0f)}
                           : motion_gradients(u, idx, i, j, dimx, dimy, P);
        // (v - dudx*v.x) - dudy*v.y
        const float2 r = make_float2((v.x - d.dx.x * v.x) - d.dy.x * v.y,
                                     (v.y - d.dx.y * v.x) - d.dy.y * v.y);
        R[idx] = r;
        const double y = (double)r.y;
        const float q = (float)(y * y + y * y);
        m = (m < q) ? q : m;
    }
    m = block_max(m);
    if (threadIdx.x == 0 && threadIdx.y == 0) part[(long)blockIdx.y * gridDim.x + blockIdx.x] = m;
}

// maxabs = sqrt(max) (float), dt = 0.65f / maxabs; scal[0]=maxabs, scal[1]=dt
__global__ __launch_bounds__(1024) void timestep_kernel(const float *__restrict__ part, int n,
                                                        float *__restrict__ scal, FluidCtl ctl) {
    if (fluid_stopped(ctl)) return;
    float m = 0.0f;
    for (int k = threadIdx.x; k < n; k += 1024) m = (m < part[k]) ? part[k] : m;
    m = wide_max(m);
    if (threadIdx.x == 0) {
        const float maxabs = sqrtf(m);
        const float dumax = 0.65f;  // OpticalFlowFluid.h:32
        scal[0] = maxabs;
        scal[1] = dumax / maxabs;
    }
}

dim3 field_grid(int dimx, int dimy) {
    return dim3((dimx + 63) / 64, (dimy + kFieldRows - 1) / kFieldRows);
}
int increment_nblocks(int dimx, int dimy) {
    const dim3 g = field_grid(dimx, dimy);
    return int(g.x * g.y);
}

void launch_increment(const float2 *u, const float4 *vel, float2 *R, int dimx, int dimy, int P,
                      float *part, float *scal, hipStream_t st, FluidCtl ctl) {
    const dim3 g = field_grid(dimx, dimy);
    hipLaunchKernelGGL(increment_kernel, g, dim3(64, 4), 0, st, u, vel, R, dimx, dimy, P, part,
                       ctl);
    hipLaunchKernelGGL(timestep_kernel, dim3(1), dim3(1024), 0, st, part, (int)(g.x * g.y), scal,
                       ctl);
    OF2D_HIP(hipGetLastError());
}

// Worker workgroups of the increment behind the sweep: -1 every CU the strips
// leave, 0 a separate increment pass (an A/B build knob: -DOF2D_SOR_NCONS=n,
// tools/build_variant.sh)
#ifndef OF2D_SOR_NCONS
#define OF2D_SOR_NCONS -1
#endif
int sor_increment_workers() { return OF2D_SOR_NCONS; }

void launch_sor_increment(float4 *vb, int dimx, int dimy, int P, float mu, float lambda,
                          float omega, void *H, unsigned epoch, unsigned *ticket,
                          unsigned long long *ctr, const float2 *u, float2 *R, float *part,
                          float *scal, unsigned *status, hipStream_t st, FluidCtl ctl) {
    const int ns = sor_nstrips(dimx);
    const dim3 g = field_grid(dimx, dimy);
    const int ntiles = (int)(g.x * g.y);
    // one 256-thread workgroup per CU (a strip's or a worker's; registers
    // allow one wave per SIMD): no strip shares its CU's load path
    int dev = 0;
    OF2D_HIP(hipGetDevice(&dev));
    // per device, queried once (the launch is on the host's critical path)
    static std::atomic<int> cus[64];
    int ncu = cus[dev & 63].load(std::memory_order_relaxed);
    if (ncu == 0) {
        OF2D_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        cus[dev & 63].store(ncu, std::memory_order_relaxed);
    }
    int nwg = sor_increment_workers();
    if (nwg < 0) nwg = ncu - ns;
    nwg = std::min(nwg, (ntiles + 3) / 4);
    if (ns == 0 || dimx < 3 || dimy < 3 || nwg < 8) {  // no sweep (OpticalFlowFluid.cpp:23-24)
        launch_sor(vb, dimx, dimy, P, mu, lambda, omega, H, epoch, ticket, status, st, ctl);
        launch_increment(u, vb, R, dimx, dimy, P, part, scal, st, ctl);
        return;
    }
    const float A = 1.0f - omega;
    const float B = omega / (-6 * mu - 2 * lambda);
    const float ML = mu + lambda;
    const SorInc inc{u, R, part, ticket + 1, ctr, nwg, ntiles, (int)g.y};
    hipLaunchKernelGGL(sor_strip_kernel<true>, dim3(ns + nwg), dim3(256), 0, st, vb, dimx, dimy,
                       P, A, B, mu, ML, (v4u *)H, sor_granule_stride(dimy), epoch, nullptr, ns,
                       status, nullptr, inc, ctl);
    hipLaunchKernelGGL(timestep_kernel, dim3(1), dim3(1024), 0, st, part, ntiles, scal, ctl);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ fused iteration step
// The end of a fluid iteration and the start of the next in one pass over a
// 64 x 32 tile (ImageRegistrationFluid.cpp:96-108, OpticalFlowFluid.cpp:97-139):
//   un = u + R dt when dt < 65, else u (OpticalFlowFluid.cpp:115),
//   written to another buffer (the halo of a neighbouring tile reads u);
//   Logger partials against prev (Logger.cpp:34-42) where prev is the Logger's
//   previous motion: the u this pass read (every iteration that follows an
//   iteration without regridding) or, kPrev, a separate field;
//   per-block min of the Jacobian of the new u (Image.cpp:189-218, Image::min
//   at Image.cpp:96-104; the neighbours' new u from an LDS tile with a
//   one-pixel halo);
//   the next iteration's force f = dI ((It + u.x dI.x) + u.y dI.y) into vb's b
//   and the region-0 granules tagged with the next sweep's epoch (sor_pack's
//   force-only mode).  When the iteration regrids, the host discards the packed
//   force and packs again.  One pass instead of three (integrate + Logger,
//   Jacobian, pack: 69 instead of 101 B/px), and no prev read or write in the
//   common case.
template <bool kPrev>
__global__ __launch_bounds__(256) void fluid_step_kernel(
    const float2 *__restrict__ u, const float2 *__restrict__ R, float2 *__restrict__ uo,
    const float2 *__restrict__ prev,
    const float *__restrict__ scal, const float2 *__restrict__ dI, const float *__restrict__ It,
    float4 *__restrict__ vb, int dimx, int dimy, int P, v4u *__restrict__ H, unsigned epoch,
    double *__restrict__ lpart, float *__restrict__ jpart, FluidCtl ctl) {
    if (fluid_stopped(ctl)) return;
    // the zero estimate of a regrid: integrated from +0, while the buffer's
    // content (the pre-regrid estimate) is the Logger's prev
    const bool zu = fluid_zero_est(ctl);
    constexpr int TW = kSkI + 2, TH = kSkJ + 2;
    __shared__ float2 un[TH][TW];       // new u at (i0 - 1 + c, j0 - 1 + r)
    __shared__ float2 fo[kSkJ][kSkI];   // the next iteration's force
    const int i0 = blockIdx.x * kSkI, j0 = blockIdx.y * kSkJ;
    const float dt = scal[1];
    const bool integ = dt < 65.0f;  // OpticalFlowFluid.cpp:135-137
    const int tid = threadIdx.y * 64 + threadIdx.x;
    // 1. new u over the tile and its one-pixel cross halo (corners unused);
    // every load of the thread is issued before the first is used (slots
    // outside the image read element 0 and are not stored)
    constexpr int NS = (TW * TH + 255) / 256;
    float2 mu[NS], mr[NS];
    bool okq[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) {
        const int s = tid + 256 * q, r = s / TW, c = s - r * TW;
        const int i = i0 - 1 + c, j = j0 - 1 + r;
        const bool corner = (r == 0 || r == TH - 1) && (c == 0 || c == TW - 1);
        okq[q] = s < TW * TH && !corner && (unsigned)i < (unsigned)dimx &&
                 (unsigned)j < (unsigned)dimy;
        const unsigned idx = okq[q] ? ((unsigned)j * (unsigned)P + (unsigned)i) : 0u;
        mu[q] = u[idx];
        mr[q] = R[idx];
    }
#pragma unroll
    for (int q = 0; q < NS; q++) {
        const int s = tid + 256 * q, r = s / TW, c = s - r * TW;
        float2 m = zu ? make_float2(0.0f, 0.0f) : mu[q];
        if (integ) m = make_float2(m.x + mr[q].x * dt, m.y + mr[q].y * dt);
        if (okq[q]) un[r][c] = m;
    }
    // 2. per pixel; thread (x, y) sums the Logger terms of rows y, y + 4, ...
    // in order; its loads first
    constexpr int NK = kSkJ / 4;
    const int i = i0 + threadIdx.x;
    float2 pvk[NK], gk[NK];
    float itk[NK];
    bool okk[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) {
        const int j = j0 + 4 * k + threadIdx.y;
        okk[k] = i < dimx && j < dimy;
        const unsigned idx = okk[k] ? ((unsigned)j * (unsigned)P + (unsigned)i) : 0u;
        pvk[k] = kPrev ? prev[idx] : u[idx];
        gk[k] = dI[idx];
        itk[k] = It[idx];
    }
    __syncthreads();
    double sd = 0.0, sp = 0.0;
    float jm = __builtin_inff();
#pragma unroll
    for (int k = 0; k < NK; k++) {
        if (!okk[k]) continue;
        const int rr = 4 * k + threadIdx.y;
        const int j = j0 + rr;
        const long idx = (long)j * P + i;
        const int r = rr + 1, c = threadIdx.x + 1;
        const float2 m = un[r][c];
        const float2 pv = pvk[k];
        uo[idx] = m;
        const float ex = m.x - pv.x, ey = m.y - pv.y;
        sd += (double)__builtin_sqrtf(ex * ex + ey * ey);
        sp += (double)__builtin_sqrtf(pv.x * pv.x + pv.y * pv.y);
        // motion_gradients of the new u (gradients.h:9-32)
        float2 dx, dy;
        if (i == 0) {
            const float2 a = un[r][c + 1], b = m;
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else if (i == dimx - 1) {
            const float2 a = m, b = un[r][c - 1];
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = un[r][c + 1], b = un[r][c - 1];
            dx = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        if (j == 0) {
            const float2 a = un[r + 1][c], b = m;
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else if (j == dimy - 1) {
            const float2 a = m, b = un[r - 1][c];
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = un[r + 1][c], b = un[r - 1][c];
            dy = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        const float q = (1.0f + dx.x) * (1.0f + dy.y) - dx.y * dy.x;  // Image.cpp:189-218
        jm = (q < jm) ? q : jm;
        // OpticalFlow::get_force (OpticalFlow.cpp:15-39) of the new u
        const float2 g = gk[k];
        const float sc = (itk[k] + m.x * g.x) + m.y * g.y;
        fo[rr][threadIdx.x] = make_float2(g.x * sc, g.y * sc);
        if (i == 0 && H) {  // ghost column of strip 0 for the next sweep
            const float2 x = reinterpret_cast<const float2 *>(vb)[sor_v(0, j, P)];
            H[kSorPadRows + j] = v4u{__float_as_uint(x.x), __float_as_uint(x.y), epoch, epoch};
        }
    }
    block_sum2(sd, sp, lpart);
    jm = block_min(jm);
    if (threadIdx.x == 0 && threadIdx.y == 0) jpart[(long)blockIdx.y * gridDim.x + blockIdx.x] = jm;
    // 3. vb's b <- force along the skewed rows
    skew_tile_set_b(vb, i0, j0, dimx, dimy, P, [&](int ii, int jj) { return fo[jj][ii]; });
}

void launch_fluid_step(const float2 *u, const float2 *R, float2 *uo, const float2 *prev,
                       const float *scal,
                       const float2 *dI, const float *It, float4 *vb, int dimx, int dimy, int P,
                       void *H, unsigned epoch, double *lpart, float *jpart, hipStream_t st,
                       FluidCtl ctl) {
    const dim3 g = field_grid(dimx, dimy);
    if (prev)
        hipLaunchKernelGGL(fluid_step_kernel<true>, g, dim3(64, 4), 0, st, u, R, uo, prev, scal,
                           dI, It, vb, dimx, dimy, P, (v4u *)H, epoch, lpart, jpart, ctl);
    else
        hipLaunchKernelGGL(fluid_step_kernel<false>, g, dim3(64, 4), 0, st, u, R, uo, prev, scal,
                           dI, It, vb, dimx, dimy, P, (v4u *)H, epoch, lpart, jpart, ctl);
    OF2D_HIP(hipGetLastError());
}

// one 1024-thread block: the Logger sums in reduce_partials_kernel's order
// (strided per-thread sums, wave trees, the 16 waves in order), the Jacobian
// minimum as min_final_kernel, then the report to host memory
__global__ __launch_bounds__(1024) void fluid_report_kernel(const double *__restrict__ p, int nb,
                                                            const float *__restrict__ jpart,
                                                            float *__restrict__ scal,
                                                            const unsigned *__restrict__ status,
                                                            FluidReport *__restrict__ rep) {
    double a = 0.0, b = 0.0;
    float m = __builtin_inff();
    for (int i = threadIdx.x; i < nb; i += 1024) {
        a += p[2 * i];
        b += p[2 * i + 1];
        m = (jpart[i] < m) ? jpart[i] : m;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    __shared__ double red[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wave] = a;
        red[1][wave] = b;
    }
    m = wide_min(m);  // (synchronises the block)
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; w++) {
            a += red[0][w];
            b += red[1][w];
        }
        scal[2] = m;
        rep->sums[0] = a;
        rep->sums[1] = b;
        rep->maxabs = scal[0];
        rep->dt = scal[1];
        rep->jmin = m;
        rep->status = *status;
    }
}

void launch_fluid_report(const double *lpart, int nb, const float *jpart, float *scal,
                         const unsigned *status, FluidReport *report, hipStream_t st) {
    hipLaunchKernelGGL(fluid_report_kernel, dim3(1), dim3(1024), 0, st, lpart, nb, jpart, scal,
                       status, report);
    OF2D_HIP(hipGetLastError());
}

// fluid_report_kernel's reductions and report, then the iteration's decisions
// as the host loop took them (ImageRegistrationFluid.cpp:99-124 with
// Logger::update_error, Logger.cpp:32-51): err = diffnorm / prevnorm in float
// (Registration's logger_error) from the exact float sums or the fp64 sums;
// break when !fixed && err < 0.001f && it > 1 (the stop word: every later
// iteration's kernels return at once); otherwise regrid when the minimum
// Jacobian is below 0.5 (kFluidRegridWord, and the motion index flips to the
// field the regrid writes).  The report's flags word is written last.
__global__ __launch_bounds__(1024) void fluid_report_decide_kernel(
    const double *__restrict__ p, int nb, const float *__restrict__ jpart,
    float *__restrict__ scal, const float *__restrict__ seq, float npx, int fixed,
    FluidReport *__restrict__ rep, FluidCtl ctl) {
    if (fluid_stopped(ctl)) return;
    double a = 0.0, b = 0.0;
    float m = __builtin_inff();
    for (int i = threadIdx.x; i < nb; i += 1024) {
        a += p[2 * i];
        b += p[2 * i + 1];
        m = (jpart[i] < m) ? jpart[i] : m;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    __shared__ double red[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wave] = a;
        red[1][wave] = b;
    }
    m = wide_min(m);  // (synchronises the block)
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; w++) {
            a += red[0][w];
            b += red[1][w];
        }
        scal[2] = m;
        // Logger::update_error's two norms as floats (logger_error: the fp64
        // sums rounded to float, or the reference's float running sums)
        const float sd = seq ? seq[0] : (float)a, sp = seq ? seq[1] : (float)b;
        const float prevnorm = sp / npx, diffnorm = sd / npx;
        const float err = prevnorm == 0.0f ? 0.0f : diffnorm / prevnorm;
        const bool brk = !fixed && err < 0.001f && ctl.it > 1;
        const bool regrid = !brk && m < 0.5f;
        unsigned *w = ctl.w;
        if (brk) atomicMin(reinterpret_cast<int *>(w + kStopWord), ctl.it);
        w[kFluidRegridWord] = regrid ? 1u : 0u;
        if (regrid) w[kFluidMcurWord] ^= 1u;
        rep->sums[0] = a;
        rep->sums[1] = b;
        rep->maxabs = scal[0];
        rep->dt = scal[1];
        rep->jmin = m;
        rep->status = w[0];
        rep->seq[0] = sd;
        rep->seq[1] = sp;
        rep->err = err;
        __atomic_store_n(&rep->flags,
                         kFluidDone | (brk ? kFluidBreak : 0u) | (regrid ? kFluidRegrid : 0u),
                         __ATOMIC_RELEASE);
    }
}
void launch_fluid_report_decide(const double *lpart, int nb, const float *jpart, float *scal,
                                const float *seq, double npx, bool fixed, FluidReport *report,
                                hipStream_t st, FluidCtl ctl) {
    if (!ctl.w) throw std::invalid_argument("launch_fluid_report_decide: control words");
    hipLaunchKernelGGL(fluid_report_decide_kernel, dim3(1), dim3(1024), 0, st, lpart, nb, jpart,
                       scal, seq, (float)npx, fixed ? 1 : 0, report, ctl);
    OF2D_HIP(hipGetLastError());
}

// Logger only (Elastic, whose update is the in-place sweep): u <- vb's v, partials
// of ||u - prev||, ||prev||; prev <- u
__global__ __launch_bounds__(256) void logger_kernel(const float4 *__restrict__ vb,
                                                     float2 *__restrict__ u,
                                                     float2 *__restrict__ prev, int dimx,
                                                     int dimy, int P,
                                                     double *__restrict__ partial) {
    __shared__ float2 vt[kSkJ][kSkI];  // as increment_kernel
    const int i0 = blockIdx.x * kSkI, j0 = blockIdx.y * kFieldRows;
    skew_tile_for_each(i0, j0, dimx, dimy, [&](int ii, int jj) {
        vt[jj][ii] = reinterpret_cast<const float2 *>(vb)[sor_v(i0 + ii, j0 + jj, P)];
    });
    __syncthreads();
    const int i = i0 + threadIdx.x;
    double sd = 0.0, sp = 0.0;
    for (int k = 0; k < kFieldRows / 4; k++) {
        const int j = j0 + 4 * k + threadIdx.y;
        if (i >= dimx || j >= dimy) break;
        const long idx = (long)j * P + i;
        const float2 m = vt[4 * k + threadIdx.y][threadIdx.x], pv = prev[idx];
        u[idx] = m;
        const float ex = m.x - pv.x, ey = m.y - pv.y;
        sd += (double)__builtin_sqrtf(ex * ex + ey * ey);
        sp += (double)__builtin_sqrtf(pv.x * pv.x + pv.y * pv.y);
        prev[idx] = m;
    }
    block_sum2(sd, sp, partial);
}
void launch_logger(const float4 *vb, float2 *u, float2 *prev, int dimx, int dimy, int P,
                   double *partial, hipStream_t st) {
    hipLaunchKernelGGL(logger_kernel, field_grid(dimx, dimy), dim3(64, 4), 0, st,
                       vb, u, prev, dimx, dimy, P, partial);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
