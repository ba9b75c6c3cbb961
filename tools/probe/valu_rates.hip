// Micro-probe (round 4): issue throughput of the integer VALU forms the
// native tier emits, on gfx950.  Each kernel runs C independent chains of one
// op per thread (8 ops per chain per inline-asm block, so no compiler s_nop
// falls between them), at W waves per SIMD (blocks of 256 = one wave per
// SIMD, 256 x W blocks).  Prints lane-ops/s per (op, C, W) as JSON lines.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/valu_rates.hip -o /tmp/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k_add_u32_vop2_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %0, 1, %0" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_add_u32_vop2_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_add_u32_vop2_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\tv_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_sub_clamp_vop3_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_sub_clamp_vop3_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_sub_clamp_vop3_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp\n\tv_sub_u32_e64 %0, %0, 1 clamp\n\tv_sub_u32_e64 %1, %1, 1 clamp\n\tv_sub_u32_e64 %2, %2, 1 clamp\n\tv_sub_u32_e64 %3, %3, 1 clamp" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_med3_i32_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %0, %0, 0, 1" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_med3_i32_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_med3_i32_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1\n\tv_med3_i32 %0, %0, 0, 1\n\tv_med3_i32 %1, %1, 0, 1\n\tv_med3_i32 %2, %2, 0, 1\n\tv_med3_i32 %3, %3, 0, 1" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_mad_i32_i24_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_mad_i32_i24_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_mad_i32_i24_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1\n\tv_mad_i32_i24 %0, %0, 3, 1\n\tv_mad_i32_i24 %1, %1, 3, 1\n\tv_mad_i32_i24 %2, %2, 3, 1\n\tv_mad_i32_i24 %3, %3, 3, 1" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_min_u32_vop2_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %0, 7, %0" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_min_u32_vop2_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_min_u32_vop2_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3\n\tv_min_u32 %0, 7, %0\n\tv_min_u32 %1, 7, %1\n\tv_min_u32 %2, 7, %2\n\tv_min_u32 %3, 7, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_pk_sub_u16_clamp_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_pk_sub_u16_clamp_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_pk_sub_u16_clamp_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp\n\tv_pk_sub_u16 %0, %0, 1 clamp\n\tv_pk_sub_u16 %1, %1, 1 clamp\n\tv_pk_sub_u16 %2, %2, 1 clamp\n\tv_pk_sub_u16 %3, %3, 1 clamp" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}
__global__ void __launch_bounds__(256) k_lshl_add_u32_1(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 1 + 0];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %0, %0, 1, %0" : "+v"(x0));
    }
    out[gid] = x0;
}
__global__ void __launch_bounds__(256) k_lshl_add_u32_2(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 2 + 0]; int x1 = in[gid * 2 + 1];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1" : "+v"(x0), "+v"(x1));
    }
    out[gid] = x0 + x1;
}
__global__ void __launch_bounds__(256) k_lshl_add_u32_4(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x0 = in[gid * 4 + 0]; int x1 = in[gid * 4 + 1]; int x2 = in[gid * 4 + 2]; int x3 = in[gid * 4 + 3];
    for (int it = 0; it < iters; it += 8) {
        __asm__ volatile("v_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3\n\tv_lshl_add_u32 %0, %0, 1, %0\n\tv_lshl_add_u32 %1, %1, 1, %1\n\tv_lshl_add_u32 %2, %2, 1, %2\n\tv_lshl_add_u32 %3, %3, 1, %3" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    out[gid] = x0 + x1 + x2 + x3;
}

typedef void (*kfn)(const int *, int *, int);
struct K { const char *name; int chains; kfn fn; };
static const K kernels[] = {
    {"add_u32_vop2", 1, k_add_u32_vop2_1},
    {"add_u32_vop2", 2, k_add_u32_vop2_2},
    {"add_u32_vop2", 4, k_add_u32_vop2_4},
    {"sub_clamp_vop3", 1, k_sub_clamp_vop3_1},
    {"sub_clamp_vop3", 2, k_sub_clamp_vop3_2},
    {"sub_clamp_vop3", 4, k_sub_clamp_vop3_4},
    {"med3_i32", 1, k_med3_i32_1},
    {"med3_i32", 2, k_med3_i32_2},
    {"med3_i32", 4, k_med3_i32_4},
    {"mad_i32_i24", 1, k_mad_i32_i24_1},
    {"mad_i32_i24", 2, k_mad_i32_i24_2},
    {"mad_i32_i24", 4, k_mad_i32_i24_4},
    {"min_u32_vop2", 1, k_min_u32_vop2_1},
    {"min_u32_vop2", 2, k_min_u32_vop2_2},
    {"min_u32_vop2", 4, k_min_u32_vop2_4},
    {"pk_sub_u16_clamp", 1, k_pk_sub_u16_clamp_1},
    {"pk_sub_u16_clamp", 2, k_pk_sub_u16_clamp_2},
    {"pk_sub_u16_clamp", 4, k_pk_sub_u16_clamp_4},
    {"lshl_add_u32", 1, k_lshl_add_u32_1},
    {"lshl_add_u32", 2, k_lshl_add_u32_2},
    {"lshl_add_u32", 4, k_lshl_add_u32_4},
};

int main()
{
    const int iters = 1 << 14;
    const int maxw = 8, threads_max = 256 * 256 * maxw;
    int *in, *out;
    if (hipMalloc(&in, sizeof(int) * threads_max * 4) != hipSuccess || hipMalloc(&out, sizeof(int) * threads_max) != hipSuccess)
        return 1;
    (void)hipMemset(in, 0, sizeof(int) * threads_max * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (const K &k : kernels) {
        for (int w = 1; w <= 8; ++w) {
            const int blocks = 256 * w;
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, in, out, iters); // warm
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, in, out, iters);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 2;
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double lane_ops = (double)blocks * 256.0 * iters * k.chains;
            printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"us\": %.2f, \"T_lane_ops\": %.2f}\n",
                   k.name, k.chains, w, ms * 1e3, lane_ops / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
