// Issue cost of the VALU instructions the traversal uses, on gfx950 (measurement tool).
// Each kernel runs a dependent-free stream of one instruction kind; 8 independent chains
// per lane, many waves per SIMD.  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_ITER 4096
#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void k(double* out, float* outf, double a, double b) {
    double x[CHAINS];
    float f[CHAINS];
    int iv[CHAINS];
    for (int c = 0; c < CHAINS; ++c) { x[c] = a + threadIdx.x + c; f[c] = (float)x[c]; iv[c] = threadIdx.x + c; }
    const unsigned long long mask = __ballot(threadIdx.x & 1);
    asm volatile("s_mov_b64 vcc, %0" :: "s"(mask) : "vcc");
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            if (OP == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[c]) : "v"(b));
            if (OP == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[c]) : "v"(b));
            if (OP == 2) asm volatile("v_min_f64 %0, %0, %1" : "+v"(x[c]) : "v"(b));
            if (OP == 3) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x[c]) : "v"(b));
            if (OP == 4) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(x[c]) : "v"(f[c]));
            if (OP == 5) asm volatile("v_cmp_lt_f64 vcc, %0, %1" :: "v"(x[c]), "v"(b) : "vcc");
            if (OP == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(iv[c]) : "v"(f[c]));
            if (OP == 14) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(iv[c]) : "v"(f[c]), "s"(mask));
            if (OP == 7) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(iv[c]) : "v"(f[c]));
            if (OP == 9) asm volatile("v_rcp_f64 %0, %0" : "+v"(x[c]));
            if (OP == 10) asm volatile("v_cmp_lt_f64 %0, %1, %2" : "=s"(*(unsigned long long*)&iv[0]) : "v"(x[c]), "v"(b));
            if (OP == 11) asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(x[c]));
            if (OP == 12) asm volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 13) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 15) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 16) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 17) asm volatile("v_min_u32 %0, %0, %1" : "+v"(iv[c]) : "v"(f[c]));
            if (OP == 18) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(f[c]) : "v"(iv[c]));
            if (OP == 19) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(x[c]));
            if (OP == 20) asm volatile("v_cmp_lt_f32 vcc, %0, %1" :: "v"(f[c]), "v"((float)b) : "vcc");
            if (OP == 21) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 22) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"((float)b), "s"((float)a));
            if (OP == 23) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"((float)b));
            if (OP == 24) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(x[c]));
            if (OP == 25) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[c]) : "v"((float)b));
        }
    }
    double s = 0;
    float sf = 0;
    for (int c = 0; c < CHAINS; ++c) { s += x[c]; sf += f[c] + iv[c]; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    outf[blockIdx.x * blockDim.x + threadIdx.x] = sf;
}
template <int OP>
void run(const char* name, double* o, float* of) {
    const int blocks = 256 * 8;   // 8 blocks of 4 waves per CU = 8 waves per SIMD
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, of, 1.0, 1e-300);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, o, of, 1.0, 1e-300);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr_per_simd = 5.0 * (blocks * 4.0 / 1024.0) * N_ITER * CHAINS;
    printf("%-16s %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n", name,
           ms * 1e6 / wave_instr_per_simd, ms * 1e6 / wave_instr_per_simd * 2.4);
}
int main() {
    double* o; float* of;
    hipMalloc(&o, 256 * 8 * 256 * 8 * 8); hipMalloc(&of, 256 * 8 * 256 * 4 * 8);
    run<0>("v_add_f64", o, of); run<1>("v_mul_f64", o, of); run<2>("v_min_f64", o, of);
    run<3>("v_fma_f64", o, of); run<4>("v_cvt_f64_f32", o, of); run<5>("v_cmp_f64(vcc)", o, of);
    run<6>("v_cndmask_b32", o, of); run<7>("v_add_f32", o, of); run<8>("v_add_u32", o, of);
    run<9>("v_rcp_f64", o, of); run<10>("v_cmp_f64(sgpr)", o, of); run<11>("v_pk_add_f32", o, of);
    run<12>("v_max_f32", o, of); run<13>("v_fma_f32", o, of); run<14>("v_cndmask(sgpr)", o, of);
    run<15>("v_min3_f32", o, of); run<16>("v_max3_f32", o, of); run<17>("v_min_u32", o, of);
    run<18>("v_cvt_f32_ubyte1", o, of); run<19>("v_pk_fma_f32", o, of); run<20>("v_cmp_f32(vcc)", o, of);
    run<21>("v_min_f32", o, of); run<22>("v_fma_f32(sgpr)", o, of); run<23>("v_med3_f32", o, of);
    run<24>("v_cvt_f32_f64", o, of); run<25>("v_mul_f32", o, of);
    return 0;
}
