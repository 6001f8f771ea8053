// valu_probe.hip — issue cost of packed vs scalar fp32 VALU on gfx950 for one
// wave alone and for four waves on one SIMD (not part of the product): loops
// of independent and dependent v_add_f32 / v_pk_add_f32 / v_pk_mul_f32 /
// v_mov_b32_dpp and fp64 add / mul / rsq / rndne in inline asm, cycles from s_memtime per instruction.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

#define REP8(x) x x x x x x x x

template <int MODE>
__global__ void probe(float *out, long long *cyc, int iters) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
          a6 = a0 + 6, a7 = a0 + 7;
    v2f p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
    const v2f k = {1e-7f, 2e-7f};
    const float kk = 1e-7f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if constexpr (MODE == 0) {  // 8 independent scalar adds x 8
            REP8(asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(kk));)
        } else if constexpr (MODE == 1) {  // 4 independent packed adds x 16 (same flops)
            REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4\n v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                         : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)
                         : "v"(k));)
        } else if constexpr (MODE == 2) {  // dependent scalar chain
            REP8(asm volatile("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1"
                         : "+v"(a0) : "v"(kk));)
        } else if constexpr (MODE == 3) {  // dependent packed chain
            REP8(asm volatile("v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %0, %0, %1"
                         : "+v"(p0) : "v"(k));)
        } else if constexpr (MODE == 4) {  // independent packed muls
            REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4\n v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                         : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)
                         : "v"(k));)
        } else if constexpr (MODE == 5) {  // independent dpp movs
            REP8(asm volatile("v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %4, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %5, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %7, %8 wave_shr:1 row_mask:0xf bank_mask:0xf"
                         : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)
                         : "v"(kk));)
        } else if constexpr (MODE == 6) {  // scalar add with the DPP shift folded into src0
            REP8(asm volatile("v_add_f32_dpp %0, %8, %0 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %1, %8, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %2, %8, %2 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %3, %8, %3 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %4, %8, %4 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %5, %8, %5 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %6, %8, %6 wave_shr:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %7, %8, %7 wave_shr:1 row_mask:0xf bank_mask:0xf"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(kk));)
        } else if constexpr (MODE >= 7) {  // fp64: 8 independent ops x 8
            double d0 = a0, d1 = a1, d2 = a2, d3 = a3;
            const double dk = 1e-9;
#define F64X8(op) REP8(asm volatile(op " %0, %0, %4\n " op " %1, %1, %4\n " op " %2, %2, %4\n " op " %3, %3, %4\n " op " %0, %0, %4\n " op " %1, %1, %4\n " op " %2, %2, %4\n " op " %3, %3, %4" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(dk));)
#define F64U8(op) REP8(asm volatile(op " %0, %0\n " op " %1, %1\n " op " %2, %2\n " op " %3, %3\n " op " %0, %0\n " op " %1, %1\n " op " %2, %2\n " op " %3, %3" : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));)
            if constexpr (MODE == 7) { F64X8("v_add_f64") }
            else if constexpr (MODE == 8) { F64X8("v_mul_f64") }
            else if constexpr (MODE == 9) { F64U8("v_rsq_f64") }
            else if constexpr (MODE == 10) { F64U8("v_rndne_f64") }
            a0 += (float)(d0 + d1 + d2 + d3);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int waves, float *out, long long *cyc) {
    const int iters = 2000;
    hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, iters);
    long long h[16];
    hipMemcpy(h, cyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    long long mx = 0;
    for (int w = 0; w < waves; w++) mx = h[w] > mx ? h[w] : mx;
    // s_memtime counts the shader clock; 64 instructions per loop iteration
    printf("%-44s waves/block %2d: %6.2f clk per instruction per wave\n", name, waves,
           (double)mx / (iters * 64.0));
}

int main() {
    float *out;
    long long *cyc;
    hipMalloc(&out, 4096 * 4);
    hipMalloc(&cyc, 64 * 8);
    for (int w : {1, 4, 16}) {
        run<0>("v_add_f32 independent", w, out, cyc);
        run<1>("v_pk_add_f32 independent", w, out, cyc);
        run<4>("v_pk_mul_f32 independent", w, out, cyc);
        run<2>("v_add_f32 dependent chain", w, out, cyc);
        run<3>("v_pk_add_f32 dependent chain", w, out, cyc);
        run<5>("v_mov_b32_dpp wave_shr independent", w, out, cyc);
        run<6>("v_add_f32_dpp wave_shr (folded) independent", w, out, cyc);
        run<7>("v_add_f64 independent", w, out, cyc);
        run<8>("v_mul_f64 independent", w, out, cyc);
        run<9>("v_rsq_f64 independent", w, out, cyc);
        run<10>("v_rndne_f64 independent", w, out, cyc);
    }
    return 0;
}
