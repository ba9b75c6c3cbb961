// Micro-probe: throughput of the C5 countdown loop shape on gfx950, full
// lanes, 8 waves per SIMD.  Variants of one iteration:
//   mask1/2/4  x -= flag; flag = x > 0   (flag a lane mask: v_subbrev + v_cmp),
//              1, 2 or 4 independent chains per thread;
//   int_med3   flag an int 0/1: x -= f; f = med3(x, 0, 1);
//   int_shift  flag an int 0/1: x -= f; f = (uint)(-x) >> 31.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void __launch_bounds__(256) chains(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x[C];
    bool a[C];
    for (int c = 0; c < C; ++c) x[c] = in[gid * C + c] + (1 << 28), a[c] = true;
    for (int it = 0; it < iters; it += 32) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                x[c] = (int)((unsigned)x[c] - (unsigned)a[c]);
                a[c] = x[c] > 0;
            }
        }
        if (__ballot(a[0]) == 0) break;
    }
    int s = 0;
    for (int c = 0; c < C; ++c) s += x[c];
    out[gid] = s;
}

template <int V>
__global__ void __launch_bounds__(256) intflag(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x = in[gid] + (1 << 28), f = 1;
    for (int it = 0; it < iters; it += 32) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            x = (int)((unsigned)x - (unsigned)f);
            // inline asm keeps LLVM from turning the 0/1 int back into a lane mask
            if (V == 0) __asm__("v_med3_i32 %0, %1, 0, 1" : "=v"(f) : "v"(x));
            else __asm__("v_sub_u32 %0, 0, %1\n\tv_lshrrev_b32 %0, 31, %0" : "=&v"(f) : "v"(x));
        }
        if (__ballot(f != 0) == 0) break;
    }
    out[gid] = x;
}

// int_fused: the bump and the flag in one asm block (no compiler s_nop
// between them); int_med3x2: two independent int-flag chains per thread.
template <int C>
__global__ void __launch_bounds__(256) intfused(const int *in, int *out, int iters)
{
    const int gid = blockIdx.x * 256 + threadIdx.x;
    int x[C], f[C];
    for (int c = 0; c < C; ++c) x[c] = in[gid * C + c] + (1 << 28), f[c] = 1;
    for (int it = 0; it < iters; it += 32) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
#pragma unroll
            for (int c = 0; c < C; ++c)
                __asm__("v_sub_u32 %0, %0, %1\n\tv_med3_i32 %1, %0, 0, 1" : "+v"(x[c]), "+v"(f[c]));
        }
        if (__ballot(f[0] != 0) == 0) break;
    }
    int s = 0;
    for (int c = 0; c < C; ++c) s += x[c];
    out[gid] = s;
}

int main()
{
    const int threads = 256 * 256 * 8; // 8 waves per SIMD on 256 CUs
    const int iters = 4096;
    int *in, *out;
    (void)hipMalloc(&in, sizeof(int) * threads * 4);
    (void)hipMalloc(&out, sizeof(int) * threads);
    (void)hipMemset(in, 0, sizeof(int) * threads * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, int C, const char *name) {
        kern<<<threads / 256, 256>>>(in, out, iters);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) kern<<<threads / 256, 256>>>(in, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double lane_iters = 5.0 * threads * (double)iters * C;
        printf("%-10s %.3f ms per launch  %.2f T lane-iterations/s\n", name, ms / 5, lane_iters / (ms * 1e-3) / 1e12);
    };
    run(chains<1>, 1, "mask1");
    run(chains<2>, 2, "mask2");
    run(chains<4>, 4, "mask4");
    run(intflag<0>, 1, "int_med3");
    run(intflag<1>, 1, "int_shift");
    run(intfused<1>, 1, "int_fused");
    run(intfused<2>, 2, "int_fusedx2");
    run(intfused<4>, 4, "int_fusedx4");
    return 0;
}
