// Where the time of a one-block call goes: an empty kernel launch + stream
// synchronisation (non-blocking stream, default stream, spin scheduling), then
// the BC4 block entry point through the library.
//   hipcc -O2 --offload-arch=gfx950 -I include tools/launch_probe.cpp -L gfx_imagecompress_amd/lib \
//         -lgfx_imagecompress_amd -o gpurun_dbg/launch_probe
//   gpurun_dbg/launch_probe [spin]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include "gfx_imagecompress/imagecompress.h"

__global__ void k_empty(int *p)
{
    if (p && threadIdx.x == 0) p[0] = 1;
}

template <class F>
static double us_per_call(int n, F f)
{
    f();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main(int argc, char **argv)
{
    if (argc > 1 && !strcmp(argv[1], "spin")) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    hipStream_t nb, bl;
    (void)hipStreamCreateWithFlags(&nb, hipStreamNonBlocking);
    (void)hipStreamCreate(&bl);
    int *d = nullptr, *h = nullptr, *hm = nullptr;
    (void)hipMalloc(&d, 4);
    (void)hipHostMalloc((void **)&h, 4, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer((void **)&hm, h, 0);
    const int n = 2000;
    printf("empty kernel, non-blocking stream sync: %8.1f us\n", us_per_call(n, [&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, nb, d);
               (void)hipStreamSynchronize(nb);
           }));
    printf("empty kernel, blocking stream sync:     %8.1f us\n", us_per_call(n, [&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, bl, d);
               (void)hipStreamSynchronize(bl);
           }));
    printf("empty kernel, null stream, device sync: %8.1f us\n", us_per_call(n, [&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, d);
               (void)hipDeviceSynchronize();
           }));
    printf("kernel writing mapped host memory:      %8.1f us\n", us_per_call(n, [&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, nb, hm);
               (void)hipStreamSynchronize(nb);
           }));
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    printf("empty kernel, event record + sync:      %8.1f us\n", us_per_call(n, [&] {
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, nb, d);
               (void)hipEventRecord(ev, nb);
               (void)hipEventSynchronize(ev);
           }));
    printf("empty kernel, poll mapped flag:         %8.1f us\n", us_per_call(n, [&] {
               *(volatile int *)h = 0;
               hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, nb, hm);
               while (*(volatile int *)h == 0) {
               }
           }));
    (void)hipStreamSynchronize(nb);
    float a16[16];
    for (int i = 0; i < 16; ++i) a16[i] = (float)((i * 37) & 15) / 15.0f;
    uint8_t out[16];
    printf("Image_CompressAMDAlphaSingleModeBlock:  %8.1f us\n",
           us_per_call(n, [&] { Image_CompressAMDAlphaSingleModeBlock(a16, out); }));
    return 0;
}
