// Micro-probe: throughput of the C5 countdown loop shape (x -= flag; flag =
// x > 0) with 1, 2 or 4 independent chains per thread, 8 waves per SIMD.
// Tells whether the predicated loop is latency- or issue-bound on gfx950.
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

int main()
{
    const int threads = 256 * 256 * 8; // 8 waves per SIMD on 256 CUs
    const int iters = 4096;
    int *in, *out;
    hipMalloc(&in, sizeof(int) * threads * 4);
    hipMalloc(&out, sizeof(int) * threads);
    hipMemset(in, 0, sizeof(int) * threads * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, int C) {
        kern<<<threads / 256, 256>>>(in, out, iters);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) kern<<<threads / 256, 256>>>(in, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double lane_iters = 5.0 * threads * (double)iters * C;
        printf("chains=%d  %.3f ms per launch  %.2f T lane-iterations/s\n", C, ms / 5, lane_iters / (ms * 1e-3) / 1e12);
    };
    run(chains<1>, 1);
    run(chains<2>, 2);
    run(chains<4>, 4);
    return 0;
}
