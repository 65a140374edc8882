// Latency of the reference-style block entry points (one block per call,
// synchronous), against the library: per-call microseconds for BC1, BC4
// (alpha single mode), BC7 (multi-mode LDR) and the BC2 colour block.
//   hipcc -O2 -I include tools/block_latency.cpp -L gfx_imagecompress_amd/lib -lgfx_imagecompress_amd -o gpurun_dbg/block_latency
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "gfx_imagecompress/imagecompress.h"

template <class F>
static double us_per_call(int n, F f)
{
    f();   // first call: allocations, table uploads
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    float blk[64], a16[16], rgb[48];
    uint32_t s = 12345;
    for (int i = 0; i < 64; ++i) {
        s = s * 1664525u + 1013904223u;
        blk[i] = (float)((s >> 8) & 255u) / 255.0f;
    }
    for (int i = 0; i < 16; ++i) a16[i] = blk[i * 4 + 3];
    for (int i = 0; i < 16; ++i)
        for (int c = 0; c < 3; ++c) rgb[i * 3 + c] = blk[i * 4 + c];
    uint8_t out[16];
    printf("BC1 block:  %8.1f us/call\n", us_per_call(n, [&] { Image_CompressAMDBC1Block(blk, false, false, 1, 0.f, out); }));
    printf("BC4 block:  %8.1f us/call\n", us_per_call(n, [&] { Image_CompressAMDAlphaSingleModeBlock(a16, out); }));
    printf("BC2 colour: %8.1f us/call\n",
           us_per_call(n, [&] { Image_CompressAMDRGBSingleModeBlock(rgb, false, false, 1, out); }));
    printf("bc7enc16:   %8.1f us/call\n", us_per_call(n, [&] { Image_CompressRichGel999BC7enc16((const uint32_t *)blk, false, true, out); }));
    printf("BC7 block:  %8.1f us/call\n",
           us_per_call(n / 10, [&] { Image_CompressAMDMultiModeLDRBlock(blk, 0xFF, true, 1.0f, false, false, 1.0f, out); }));
    return 0;
}
