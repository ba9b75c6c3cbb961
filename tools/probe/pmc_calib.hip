// pmc_calib.hip -- byte-count calibration of rocprofv3's FETCH_SIZE /
// WRITE_SIZE on gfx950 for the access pattern of the heavy kernel's stack
// slots: wave-blocked [wave][slot][64] int32, one
// 4-byte buffer load or store per lane per slot (256 B per wave
// instruction), as tis_jit.cpp's mk_slot_st / mk_slot_ld emit them.  Beside
// it the guide's calibrated case, 16 B per lane streaming loads
// (MI355X_MICROARCH.md section HBM: FETCH_SIZE reads half of those bytes).
//
//   pmc_calib MODE MIB
//     MODE = st4 | ld4 | ld16;  MIB = bytes moved per launch / 2^20
// Launches the kernel 5 times (the first two are warm-up, tools/
// pmc_calib_fold.py skips them) and prints the known byte count per launch.
// Sizes far above the 256 MiB Infinity Cache keep the counts HBM traffic.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

constexpr int kSlots = 256; // slots per wave block (a C4 d256-sized lane)

__device__ __amdgpu_buffer_rsrc_t wave_rsrc(int32_t *base)
{
    return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)(256u * kSlots), 0x00020000);
}

__global__ void __launch_bounds__(64) st4(int32_t *slots)
{
    int32_t *b = slots + (size_t)blockIdx.x * kSlots * 64u;
    const __amdgpu_buffer_rsrc_t r = wave_rsrc(b);
    const int32_t lane = (int32_t)(threadIdx.x * 4u);
    for (uint32_t s = 0; s < kSlots; ++s)
        __builtin_amdgcn_raw_buffer_store_b32((int32_t)(s ^ threadIdx.x), r, lane + (int32_t)(s * 256u), 0, 0);
}

__global__ void __launch_bounds__(64) ld4(int32_t *slots, int32_t *out)
{
    int32_t *b = slots + (size_t)blockIdx.x * kSlots * 64u;
    const __amdgpu_buffer_rsrc_t r = wave_rsrc(b);
    const int32_t lane = (int32_t)(threadIdx.x * 4u);
    int32_t acc = 0;
#pragma unroll 16
    for (uint32_t s = 0; s < kSlots; ++s)
        acc = 3 * acc + __builtin_amdgcn_raw_buffer_load_b32(r, lane + (int32_t)(s * 256u), 0, 0);
    if (acc == 0x7fffffff) out[0] = acc; // keeps the loads; never true for the data written
}

__global__ void __launch_bounds__(256) ld16(const int4 *src, int32_t *out, size_t n)
{
    int32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (size_t)gridDim.x * 256u) {
        const int4 v = src[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: pmc_calib st4|ld4|ld16 MIB\n");
        return 2;
    }
    const char *mode = argv[1];
    const size_t bytes = (size_t)std::strtoull(argv[2], nullptr, 10) << 20;
    const size_t wave_bytes = (size_t)kSlots * 256u;
    const unsigned waves = (unsigned)(bytes / wave_bytes);
    const size_t used = (size_t)waves * wave_bytes;
    if (waves == 0) return 2;
    int32_t *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, used) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, used) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms_total = 0.f;
    for (int it = 0; it < 5; ++it) {
        (void)hipEventRecord(a, 0);
        if (!std::strcmp(mode, "st4")) hipLaunchKernelGGL(st4, dim3(waves), dim3(64), 0, 0, buf);
        else if (!std::strcmp(mode, "ld4")) hipLaunchKernelGGL(ld4, dim3(waves), dim3(64), 0, 0, buf, out);
        else hipLaunchKernelGGL(ld16, dim3(4096), dim3(256), 0, 0, (const int4 *)buf, out, used / 16);
        (void)hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 1;
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (it >= 2) ms_total += ms;
    }
    std::printf("{\"mode\": \"%s\", \"bytes_per_launch\": %zu, \"waves\": %u, \"us_per_launch\": %.2f, \"GBps\": %.1f}\n",
                mode, used, waves, 1000.0 * ms_total / 3, used / (ms_total / 3 * 1e6));
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}
