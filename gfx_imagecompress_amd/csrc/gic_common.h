// gic_common.h -- shared device/host helpers for the MI355X BCn kernels.
//
// Numerics contract: every kernel translation unit is compiled with
// -ffp-contract=off (no v_fma/v_fmac contraction), correctly rounded f32
// divide/sqrt and IEEE f64, so each non-exact expression rounds exactly as
// the reference's x86-64 SSE build.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gfx_imagecompress_amd/gic.h"

namespace gic {

// Geometry of one launch: which blocks of which image it covers.
struct Geometry {
    const uint8_t *src;
    uint32_t width, height, slices, channels;
    size_t row_pitch;
    uint32_t bx_count;   // blocks per row
    uint32_t row0;       // first block row of the shard
    uint32_t nrows;      // block rows per slice in the shard
    uint32_t total;      // blocks in the launch = bx_count * nrows * slices
};

// Reference-style minimum / maximum (Math_MinF / Math_MaxF are a<b?a:b).
__device__ __forceinline__ float minr(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float maxr(float a, float b) { return a > b ? a : b; }

// Decompose a linear block id of a launch into (slice, block row, block col).
__device__ __forceinline__ void block_coords(const Geometry &g, uint32_t id, uint32_t &slice,
                                             uint32_t &by, uint32_t &bx)
{
    bx = id % g.bx_count;
    const uint32_t r = id / g.bx_count;
    by = g.row0 + r % g.nrows;
    slice = r / g.nrows;
}

// Gather the 4x4 texels of a block as float RGBA in [0,1] (v / 255.0f),
// replicating the last row/column past the image edge (ReadNxNBlockF,
// block_utils.cpp:7-41).  Interior RGBA8 blocks use four 16-byte row loads:
// adjacent lanes hold adjacent blocks, so each row is one coalesced 1 KiB
// wave access.
__device__ __forceinline__ void load_block(const Geometry &g, uint32_t slice, uint32_t by, uint32_t bx,
                                           bool force_alpha_one, float out[64])
{
    const uint8_t *img = g.src + (size_t)slice * g.row_pitch * g.height;
    const uint32_t x0 = bx * 4, y0 = by * 4;
    if (g.channels == 4 && x0 + 4 <= g.width && y0 + 4 <= g.height && (g.row_pitch & 15) == 0 &&
        ((uintptr_t)g.src & 15) == 0) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint4 row = *reinterpret_cast<const uint4 *>(img + (size_t)(y0 + y) * g.row_pitch + x0 * 4);
            const uint32_t w[4] = {row.x, row.y, row.z, row.w};
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    out[(y * 4 + x) * 4 + c] = (float)((w[x] >> (8 * c)) & 0xffu) / 255.0f;
        }
    } else {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            uint32_t sy = y0 + y;
            sy = sy >= g.height ? g.height - 1 : sy;
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                uint32_t sx = x0 + x;
                sx = sx >= g.width ? g.width - 1 : sx;
                const uint8_t *p = img + (size_t)sy * g.row_pitch + (size_t)sx * g.channels;
                float *o = out + (y * 4 + x) * 4;
                o[0] = (float)p[0] / 255.0f;
                o[1] = g.channels > 1 ? (float)p[1] / 255.0f : 0.f;
                o[2] = g.channels > 2 ? (float)p[2] / 255.0f : 0.f;
                o[3] = g.channels > 3 ? (float)p[3] / 255.0f : 1.f;
            }
        }
    }
    if (force_alpha_one || g.channels < 4) {
#pragma unroll
        for (int i = 0; i < 16; ++i) out[i * 4 + 3] = 1.0f;
    }
}

// The same gather as packed RGBA8 words (R | G << 8 | B << 16 | A << 24):
// missing channels read 0 (alpha 255), the float view of a byte v is v / 255.0f.
__device__ __forceinline__ void load_block_u8(const Geometry &g, uint32_t slice, uint32_t by, uint32_t bx,
                                              bool force_alpha_one, uint32_t out[16])
{
    const uint8_t *img = g.src + (size_t)slice * g.row_pitch * g.height;
    const uint32_t x0 = bx * 4, y0 = by * 4;
    if (g.channels == 4 && x0 + 4 <= g.width && y0 + 4 <= g.height && (g.row_pitch & 15) == 0 &&
        ((uintptr_t)g.src & 15) == 0) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint4 row = *reinterpret_cast<const uint4 *>(img + (size_t)(y0 + y) * g.row_pitch + x0 * 4);
            out[y * 4 + 0] = row.x;
            out[y * 4 + 1] = row.y;
            out[y * 4 + 2] = row.z;
            out[y * 4 + 3] = row.w;
        }
    } else if (g.channels == 1 && x0 + 4 <= g.width && y0 + 4 <= g.height && (g.row_pitch & 3) == 0 &&
               ((uintptr_t)g.src & 3) == 0) {
        // R8: one 4-byte load per row
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint32_t row = *reinterpret_cast<const uint32_t *>(img + (size_t)(y0 + y) * g.row_pitch + x0);
#pragma unroll
            for (int x = 0; x < 4; ++x) out[y * 4 + x] = (row >> (8 * x)) & 0xffu;
        }
    } else if (g.channels == 2 && x0 + 4 <= g.width && y0 + 4 <= g.height && (g.row_pitch & 7) == 0 &&
               ((uintptr_t)g.src & 7) == 0) {
        // R8G8: one 8-byte load per row
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint2 row = *reinterpret_cast<const uint2 *>(img + (size_t)(y0 + y) * g.row_pitch + x0 * 2);
            out[y * 4 + 0] = row.x & 0xffffu;
            out[y * 4 + 1] = row.x >> 16;
            out[y * 4 + 2] = row.y & 0xffffu;
            out[y * 4 + 3] = row.y >> 16;
        }
    } else {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            uint32_t sy = y0 + y;
            sy = sy >= g.height ? g.height - 1 : sy;
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                uint32_t sx = x0 + x;
                sx = sx >= g.width ? g.width - 1 : sx;
                const uint8_t *p = img + (size_t)sy * g.row_pitch + (size_t)sx * g.channels;
                uint32_t w = p[0];
                if (g.channels > 1) w |= (uint32_t)p[1] << 8;
                if (g.channels > 2) w |= (uint32_t)p[2] << 16;
                w |= (g.channels > 3 ? (uint32_t)p[3] : 255u) << 24;
                out[y * 4 + x] = w;
            }
        }
    }
    if (force_alpha_one || g.channels < 4) {
#pragma unroll
        for (int i = 0; i < 16; ++i) out[i] |= 0xff000000u;
    }
}

}  // namespace gic
