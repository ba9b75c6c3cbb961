// Micro-probe (round 4): the C4 pop body's chain, sum = 3 * sum + v, in the
// forms a compiler can give it, as ONE dependent chain per lane at one wave
// per SIMD (the heavy LDS kernel's occupancy) and at 8.  Values come from a
// register array (no memory), so the time is the chain's.  JSON lines:
// lane-steps/s and cycles per step per wave.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/valu_chain.hip -o tools/probe/valu_chain.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

// 64-bit mad as LLVM emits it (src0 = the low half of its own destination pair)
#define STEP_MAD64 "v_mad_u64_u32 v[100:101], vcc, v100, 3, v[102:103]\n\t"
#define STEP_LSHLADD "v_lshl_add_u32 %0, %0, 1, %0\n\tv_add_u32 %0, %0, %1\n\t"
#define STEP_ADD3 "v_add3_u32 %0, %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\t"  // s+s+v, + s_old kept in %2
#define STEP_MUL "v_mul_lo_u32 %0, %0, 3\n\tv_add_u32 %0, %0, %1\n\t"

template <int F>
__global__ void __launch_bounds__(256) chain(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    uint32_t s = in[gid], v = in[gid] ^ 5u;
    uint64_t s64 = 0;
    if (F == 0)
        __asm__ volatile("v_mov_b32 v100, %0\n\tv_mov_b32 v101, 0\n\tv_mov_b32 v102, %1\n\tv_mov_b32 v103, 0"
                         :: "v"(s), "v"(v) : "v100", "v101", "v102", "v103");
    for (int it = 0; it < iters; it += 8) {
        if (F == 0) {
            __asm__ volatile(STEP_MAD64 STEP_MAD64 STEP_MAD64 STEP_MAD64 STEP_MAD64 STEP_MAD64 STEP_MAD64 STEP_MAD64
                             ::: "v100", "v101", "v102", "v103", "vcc");
        } else if (F == 1) {
            __asm__ volatile(STEP_LSHLADD STEP_LSHLADD STEP_LSHLADD STEP_LSHLADD STEP_LSHLADD STEP_LSHLADD
                             STEP_LSHLADD STEP_LSHLADD : "+v"(s) : "v"(v));
        } else if (F == 2) {
            uint32_t t = s;
            __asm__ volatile(STEP_ADD3 STEP_ADD3 STEP_ADD3 STEP_ADD3 STEP_ADD3 STEP_ADD3 STEP_ADD3 STEP_ADD3
                             : "+v"(s) : "v"(v), "v"(t));
        } else {
            __asm__ volatile(STEP_MUL STEP_MUL STEP_MUL STEP_MUL STEP_MUL STEP_MUL STEP_MUL STEP_MUL : "+v"(s) : "v"(v));
        }
    }
    if (F == 0) {
        uint32_t r;
        __asm__ volatile("v_mov_b32 %0, v100" : "=v"(r) :: "v100");
        s64 = r;
    }
    out[gid] = (int)(s + (uint32_t)s64);
}

int main()
{
    const int iters = 1 << 14, threads_max = 256 * 256 * 8;
    int *in, *out;
    if (hipMalloc(&in, sizeof(int) * threads_max) != hipSuccess || hipMalloc(&out, sizeof(int) * threads_max) != hipSuccess)
        return 1;
    (void)hipMemset(in, 0, sizeof(int) * threads_max);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[] = {"mad_u64_u32", "lshl_add+add", "add3+add", "mul_lo+add"};
    void (*fns[])(const int *, int *, int) = {chain<0>, chain<1>, chain<2>, chain<3>};
    for (int f = 0; f < 4; ++f) {
        for (int w : {1, 2, 4, 8}) {
            const int blocks = 256 * w;
            hipLaunchKernelGGL(fns[f], dim3(blocks), dim3(256), 0, 0, in, out, iters);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(fns[f], dim3(blocks), dim3(256), 0, 0, in, out, iters);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) return 2;
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double steps = (double)blocks * 256.0 * iters;
            printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"us\": %.2f, \"T_lane_steps\": %.3f, "
                   "\"cycles_per_step_per_wave\": %.2f}\n", names[f], w, ms * 1e3, steps / (ms * 1e-3) / 1e12,
                   (ms * 1e-3) * 2.4e9 / ((double)iters * w));
            fflush(stdout);
        }
    }
    return 0;
}
