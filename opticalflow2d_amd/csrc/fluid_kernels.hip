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
//     NEW values from the previous strip through 8-byte {epoch, value}
//     granules (agent-scope release/acquire-free hand-off, MI355X guide §6
//     G16 R2), prefetched a few steps ahead; lane 63 is a ghost of the next
//     strip's first column (OLD values, which that strip cannot overwrite
//     before this strip has published the rows that depend on them);
//   * strips are claimed in order through a ticket counter, so a strip only
//     ever waits on a strip that is already running (no deadlock whatever the
//     dispatch order); every spin is bounded and reports through the status
//     word.
#include "of2d_device.h"

namespace of2d {

namespace {
constexpr int kStripCols = 62;
constexpr int kPre = 8;    // rows of OLD values prefetched ahead of the window
constexpr int kGPre = 8;   // granule rows prefetched ahead by lane 0
constexpr unsigned kSpinLimit = 1u << 24;

typedef unsigned long long u64;

__device__ __forceinline__ u64 gload(const u64 *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(u64 *p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 granule(unsigned epoch, float v) {
    return ((u64)epoch << 32) | (u64)__float_as_uint(v);
}

struct Px {  // what one lane needs at one row
    float2 v;     // OLD velocity
    float2 g;     // dI
    float2 u;     // motion (fused force) or force b
    float it;     // It (fused force)
};

template <bool FUSED>
__device__ __forceinline__ Px load_px(const float2 *v, const float2 *u, const float2 *dI,
                                      const float *It, int c, int r, int dimx, int dimy, int P) {
    Px p;
    const int cc = min(max(c, 0), dimx - 1), rr = min(max(r, 0), dimy - 1);
    const long idx = (long)rr * P + cc;
    p.v = v[idx];
    p.u = u[idx];
    if constexpr (FUSED) {
        p.g = dI[idx];
        p.it = It[idx];
    } else {
        p.g = make_float2(0.0f, 0.0f);
        p.it = 0.0f;
    }
    return p;
}

__device__ __forceinline__ float2 shfl_up2(float2 a) {
    return make_float2(__shfl_up(a.x, 1), __shfl_up(a.y, 1));
}
__device__ __forceinline__ float2 shfl_down2(float2 a) {
    return make_float2(__shfl_down(a.x, 1), __shfl_down(a.y, 1));
}
}  // namespace

// FUSED: b = force computed from (u, dI, It) of the same pixel (Fluid: u is not
// modified by the sweep).  !FUSED: b read from `u` (Elastic: the force is
// computed before the sweep and the sweep updates the motion itself).
template <bool FUSED>
__global__ __launch_bounds__(64) void sor_strip_kernel(
    float2 *__restrict__ v, const float2 *__restrict__ u, const float2 *__restrict__ dI,
    const float *__restrict__ It, int dimx, int dimy, int P, float A, float B, float M, float ML,
    u64 *__restrict__ H, unsigned epoch, unsigned *__restrict__ ticket, int nstrips,
    unsigned *__restrict__ status) {
    const int lane = threadIdx.x;
    __shared__ int s_strip;
    if (lane == 0) s_strip = (int)(atomicAdd(ticket, 1u) % (unsigned)nstrips);
    __syncthreads();
    const int I = s_strip;
    const int c0 = kStripCols * I;  // lane 0 = column c0 (previous strip's last column)
    const int c = c0 + lane;
    const bool active = lane >= 1 && lane <= kStripCols && c <= dimx - 2;
    // this strip publishes its last column when a next strip exists
    const bool publisher = (lane == kStripCols) && active && (c + 1 <= dimx - 2);
    const bool consumer = (lane == 0) && (I > 0);
    u64 *Hout = H + (size_t)I * dimy * 2;          // our column c0 + 62
    const u64 *Hin = H + (size_t)(I - 1) * dimy * 2;  // previous strip's column c0

    // row of this lane at step s: r = s - 2(lane-1) + 1 (lane 0: s + 3)
    const int rofs = 3 - 2 * lane;  // r = s + rofs
    const int s0 = -3;
    const int s1 = (dimy - 2) - 1 + 2 * (kStripCols - 1);  // last step of lane 62

    // window of OLD values rows r..r+3 and a prefetch FIFO rows r+4..r+3+kPre
    float2 w[4];
    Px fifo[kPre];
    Px cur[4];  // Px for rows r..r+3 (v, force inputs)
    {
        const int r = s0 + rofs;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            cur[k] = load_px<FUSED>(v, u, dI, It, c, r + k, dimx, dimy, P);
            w[k] = cur[k].v;
        }
#pragma unroll
        for (int k = 0; k < kPre; k++) fifo[k] = load_px<FUSED>(v, u, dI, It, c, r + 4 + k, dimx, dimy, P);
    }
    // lane 0: granule prefetch FIFO for rows q..q+kGPre-1, q = s + 3
    u64 gx[kGPre], gy[kGPre];
    if (consumer) {
#pragma unroll
        for (int k = 0; k < kGPre; k++) {
            const int q = s0 + 3 + k;
            const int qq = min(max(q, 0), dimy - 1);
            gx[k] = gload(Hin + 2 * (size_t)qq);
            gy[k] = gload(Hin + 2 * (size_t)qq + 1);
        }
    }
    float2 h1 = w[0], h2 = w[0], h3 = w[0];  // own outputs at s-1, s-2, s-3
    unsigned bad = 0;

    for (int s = s0; s <= s1; s++) {
        const int r = s + rofs;
        // ---- this lane's output at step s (before the shuffles of step s+1)
        float2 out = w[0];  // boundary rows / inactive: the OLD value
        // ---- left neighbour NEW values: its outputs at s-1, s-2, s-3
        const float2 LU = shfl_up2(h1), L = shfl_up2(h2), LD = shfl_up2(h3);
        // ---- right neighbour OLD values rows r-1, r, r+1 = its window w1..w3
        const float2 RD = shfl_down2(w[1]), R = shfl_down2(w[2]), RU = shfl_down2(w[3]);
        if (lane == 0) {
            // ghost of column c0: NEW value at row q = r
            const int q = r;
            if (consumer && q >= 1 && q <= dimy - 2) {
                u64 a = gx[0], b = gy[0];
                unsigned spins = 0;
                while ((unsigned)(a >> 32) != epoch || (unsigned)(b >> 32) != epoch) {
                    if (++spins > kSpinLimit) {
                        atomicOr(status, kStatusSpinTimeout);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    a = gload(Hin + 2 * (size_t)q);
                    b = gload(Hin + 2 * (size_t)q + 1);
                }
                out = make_float2(__uint_as_float((unsigned)a), __uint_as_float((unsigned)b));
            }
        } else if (active && r >= 1 && r <= dimy - 2) {
            const Px &p = cur[0];
            float2 b;
            if constexpr (FUSED) {
                // OpticalFlow.cpp:33: dI * (It + u.x*dI.x + u.y*dI.y)
                const float sc = (p.it + p.u.x * p.g.x) + p.u.y * p.g.y;
                b = make_float2(p.g.x * sc, p.g.y * sc);
            } else {
                b = p.u;
            }
            const float2 C = w[0], U = w[1], D = h1;
            // OpticalFlowFluid.cpp:27-35 (same association, no contraction)
            const float s1x = ((R.x + L.x) + U.x) + D.x;
            const float s2x = (R.x + L.x) + 0.25f * (((RU.y - LU.y) - RD.y) + LD.y);
            const float nx = A * C.x + B * ((b.x - M * s1x) - ML * s2x);
            const float s1y = ((R.y + L.y) + U.y) + D.y;
            const float s2y = (R.y + L.y) + 0.25f * (((RU.x - LU.x) - RD.x) + LD.x);
            const float ny = A * C.y + B * ((b.y - M * s1y) - ML * s2y);
            out = make_float2(nx, ny);
            v[(long)r * P + c] = out;
            if (publisher) {
                gstore(Hout + 2 * (size_t)r, granule(epoch, nx));
                gstore(Hout + 2 * (size_t)r + 1, granule(epoch, ny));
            }
        }
        // ---- shift histories, window and prefetch queues
        h3 = h2;
        h2 = h1;
        h1 = out;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            cur[k] = cur[k + 1];
            w[k] = w[k + 1];
        }
        cur[3] = fifo[0];
        w[3] = fifo[0].v;
#pragma unroll
        for (int k = 0; k < kPre - 1; k++) fifo[k] = fifo[k + 1];
        fifo[kPre - 1] = load_px<FUSED>(v, u, dI, It, c, r + 4 + kPre, dimx, dimy, P);
        if (consumer) {
#pragma unroll
            for (int k = 0; k < kGPre - 1; k++) {
                gx[k] = gx[k + 1];
                gy[k] = gy[k + 1];
            }
            const int qn = r + 1 + (kGPre - 1);
            const int qq = min(max(qn, 0), dimy - 1);
            gx[kGPre - 1] = gload(Hin + 2 * (size_t)qq);
            gy[kGPre - 1] = gload(Hin + 2 * (size_t)qq + 1);
        }
    }
    (void)bad;
}

int sor_nstrips(int dimx) { return dimx < 3 ? 0 : (dimx - 2 + kStripCols - 1) / kStripCols; }

void launch_sor(float2 *v, const float2 *u_or_b, const float2 *dI, const float *It, bool fused,
                int dimx, int dimy, int P, float mu, float lambda, float omega,
                unsigned long long *H, unsigned epoch, unsigned *ticket, unsigned *status,
                hipStream_t st) {
    if (dimx < 3 || dimy < 3) return;  // no interior (OpticalFlowFluid.cpp:23-24)
    const int ns = sor_nstrips(dimx);
    // per-pixel constants of OpticalFlowFluid.cpp:27 evaluated once, same float ops
    const float A = 1.0f - omega;
    const float B = omega / (-6 * mu - 2 * lambda);
    const float ML = mu + lambda;
    if (fused)
        hipLaunchKernelGGL(sor_strip_kernel<true>, dim3(ns), dim3(64), 0, st, v, u_or_b, dI, It,
                           dimx, dimy, P, A, B, mu, ML, (u64 *)H, epoch, ticket, ns, status);
    else
        hipLaunchKernelGGL(sor_strip_kernel<false>, dim3(ns), dim3(64), 0, st, v, u_or_b, dI, It,
                           dimx, dimy, P, A, B, mu, ML, (u64 *)H, epoch, ticket, ns, status);
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
                                                        const float2 *__restrict__ vel,
                                                        float2 *__restrict__ R, int dimx, int dimy,
                                                        int P, float *__restrict__ part) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    float m = 0.0f;
    if (i < dimx && j < dimy) {
        const long idx = (long)j * P + i;
        const float2 v = vel[idx];
        float2 dx, dy;
        if (i == 0) {
            const float2 a = u[idx + 1], b = u[idx];
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else if (i == dimx - 1) {
            const float2 a = u[idx], b = u[idx - 1];
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = u[idx + 1], b = u[idx - 1];
            dx = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        if (j == 0) {
            const float2 a = u[idx + P], b = u[idx];
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else if (j == dimy - 1) {
            const float2 a = u[idx], b = u[idx - P];
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = u[idx + P], b = u[idx - P];
            dy = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        // (v - dudx*v.x) - dudy*v.y
        const float2 r = make_float2((v.x - dx.x * v.x) - dy.x * v.y, (v.y - dx.y * v.x) - dy.y * v.y);
        R[idx] = r;
        const double y = (double)r.y;
        m = (float)(y * y + y * y);
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (m < o) ? o : m;
    }
    __shared__ float red[4];
    const int t = threadIdx.y * 64 + threadIdx.x;
    if ((t & 63) == 0) red[t >> 6] = m;
    __syncthreads();
    if (t == 0) {
        float a = red[0];
        for (int w = 1; w < 4; w++) a = (a < red[w]) ? red[w] : a;
        part[(long)blockIdx.y * gridDim.x + blockIdx.x] = a;
    }
}

// maxabs = sqrt(max) (float), dt = 0.65f / maxabs; scal[0]=maxabs, scal[1]=dt
__global__ void timestep_kernel(const float *__restrict__ part, int n, float *__restrict__ scal) {
    __shared__ float red[256];
    float m = 0.0f;
    for (int k = threadIdx.x; k < n; k += 256) m = (m < part[k]) ? part[k] : m;
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const float o = red[threadIdx.x + w];
            red[threadIdx.x] = (red[threadIdx.x] < o) ? o : red[threadIdx.x];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float maxabs = sqrtf(red[0]);
        const float dumax = 0.65f;  // OpticalFlowFluid.h:32
        scal[0] = maxabs;
        scal[1] = dumax / maxabs;
    }
}

int increment_nblocks(int dimx, int dimy) { return ((dimx + 63) / 64) * ((dimy + 3) / 4); }

void launch_increment(const float2 *u, const float2 *vel, float2 *R, int dimx, int dimy, int P,
                      float *part, float *scal, hipStream_t st) {
    const dim3 g((dimx + 63) / 64, (dimy + 3) / 4);
    hipLaunchKernelGGL(increment_kernel, g, dim3(64, 4), 0, st, u, vel, R, dimx, dimy, P, part);
    hipLaunchKernelGGL(timestep_kernel, dim3(1), dim3(256), 0, st, part, (int)(g.x * g.y), scal);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ integrate + Logger
// if dt < 65: u += R*dt (OpticalFlowFluid.cpp:115, skipped per :135-137); then
// Logger::update_error against `prev` (Logger.cpp:34-42): partial sums of
// ||u - prev|| and ||prev||, prev <- u.
__global__ __launch_bounds__(256) void integrate_logger_kernel(float2 *__restrict__ u,
                                                               const float2 *__restrict__ R,
                                                               float2 *__restrict__ prev,
                                                               const float *__restrict__ scal,
                                                               int dimx, int dimy, int P,
                                                               double *__restrict__ partial) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    double sd = 0.0, sp = 0.0;
    if (i < dimx && j < dimy) {
        const long idx = (long)j * P + i;
        const float dt = scal[1];
        float2 m = u[idx];
        if (dt < 65.0f) {
            const float2 r = R[idx];
            m = make_float2(m.x + r.x * dt, m.y + r.y * dt);
            u[idx] = m;
        }
        const float2 pv = prev[idx];
        const float ex = m.x - pv.x, ey = m.y - pv.y;
        sd = (double)__builtin_sqrtf(ex * ex + ey * ey);
        sp = (double)__builtin_sqrtf(pv.x * pv.x + pv.y * pv.y);
        prev[idx] = m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off);
        sp += __shfl_down(sp, off);
    }
    __shared__ double red[2][4];
    const int t = threadIdx.y * 64 + threadIdx.x;
    if ((t & 63) == 0) {
        red[0][t >> 6] = sd;
        red[1][t >> 6] = sp;
    }
    __syncthreads();
    if (t == 0) {
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        partial[2 * blk + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}

void launch_integrate_logger(float2 *u, const float2 *R, float2 *prev, const float *scal,
                             int dimx, int dimy, int P, double *partial, hipStream_t st) {
    hipLaunchKernelGGL(integrate_logger_kernel, dim3((dimx + 63) / 64, (dimy + 3) / 4),
                       dim3(64, 4), 0, st, u, R, prev, scal, dimx, dimy, P, partial);
    OF2D_HIP(hipGetLastError());
}

// Logger only (Elastic / Curvature, whose update is in place): partials of
// ||u - prev||, ||prev||; prev <- u
__global__ __launch_bounds__(256) void logger_kernel(const float2 *__restrict__ u,
                                                     float2 *__restrict__ prev, int dimx,
                                                     int dimy, int P,
                                                     double *__restrict__ partial) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    double sd = 0.0, sp = 0.0;
    if (i < dimx && j < dimy) {
        const long idx = (long)j * P + i;
        const float2 m = u[idx], pv = prev[idx];
        const float ex = m.x - pv.x, ey = m.y - pv.y;
        sd = (double)__builtin_sqrtf(ex * ex + ey * ey);
        sp = (double)__builtin_sqrtf(pv.x * pv.x + pv.y * pv.y);
        prev[idx] = m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        sd += __shfl_down(sd, off);
        sp += __shfl_down(sp, off);
    }
    __shared__ double red[2][4];
    const int t = threadIdx.y * 64 + threadIdx.x;
    if ((t & 63) == 0) {
        red[0][t >> 6] = sd;
        red[1][t >> 6] = sp;
    }
    __syncthreads();
    if (t == 0) {
        const long blk = (long)blockIdx.y * gridDim.x + blockIdx.x;
        partial[2 * blk] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        partial[2 * blk + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    }
}
void launch_logger(const float2 *u, float2 *prev, int dimx, int dimy, int P, double *partial,
                   hipStream_t st) {
    hipLaunchKernelGGL(logger_kernel, dim3((dimx + 63) / 64, (dimy + 3) / 4), dim3(64, 4), 0, st,
                       u, prev, dimx, dimy, P, partial);
    OF2D_HIP(hipGetLastError());
}

// ------------------------------------------------------------ jacobian min
// Image::jacobian (Image.cpp:189-218): (1 + dudx.x)(1 + dudy.y) - dudx.y dudy.x,
// then Image::min (Image.cpp:96-104): per-block min, final min in scal[2]
__global__ __launch_bounds__(256) void jacobian_min_kernel(const float2 *__restrict__ u,
                                                           int dimx, int dimy, int P,
                                                           float *__restrict__ part) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y * 4 + threadIdx.y;
    float m = __builtin_inff();
    if (i < dimx && j < dimy) {
        const long idx = (long)j * P + i;
        float2 dx, dy;
        if (i == 0) {
            const float2 a = u[idx + 1], b = u[idx];
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else if (i == dimx - 1) {
            const float2 a = u[idx], b = u[idx - 1];
            dx = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = u[idx + 1], b = u[idx - 1];
            dx = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        if (j == 0) {
            const float2 a = u[idx + P], b = u[idx];
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else if (j == dimy - 1) {
            const float2 a = u[idx], b = u[idx - P];
            dy = make_float2(a.x - b.x, a.y - b.y);
        } else {
            const float2 a = u[idx + P], b = u[idx - P];
            dy = make_float2((a.x - b.x) / 2.0f, (a.y - b.y) / 2.0f);
        }
        m = (1.0f + dx.x) * (1.0f + dy.y) - dx.y * dy.x;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_down(m, off);
        m = (o < m) ? o : m;
    }
    __shared__ float red[4];
    const int t = threadIdx.y * 64 + threadIdx.x;
    if ((t & 63) == 0) red[t >> 6] = m;
    __syncthreads();
    if (t == 0) {
        float a = red[0];
        for (int w = 1; w < 4; w++) a = (red[w] < a) ? red[w] : a;
        part[(long)blockIdx.y * gridDim.x + blockIdx.x] = a;
    }
}
__global__ void min_final_kernel(const float *__restrict__ part, int n, float *__restrict__ out) {
    __shared__ float red[256];
    float m = __builtin_inff();
    for (int k = threadIdx.x; k < n; k += 256) m = (part[k] < m) ? part[k] : m;
    red[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const float o = red[threadIdx.x + w];
            red[threadIdx.x] = (o < red[threadIdx.x]) ? o : red[threadIdx.x];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}
void launch_jacobian_min(const float2 *u, int dimx, int dimy, int P, float *part, float *out,
                         hipStream_t st) {
    const dim3 g((dimx + 63) / 64, (dimy + 3) / 4);
    hipLaunchKernelGGL(jacobian_min_kernel, g, dim3(64, 4), 0, st, u, dimx, dimy, P, part);
    hipLaunchKernelGGL(min_final_kernel, dim3(1), dim3(256), 0, st, part, (int)(g.x * g.y), out);
    OF2D_HIP(hipGetLastError());
}

}  // namespace of2d
