// gic_fastdiv.h -- the two float divisions of the BC1 endpoint search in a
// cheaper exact form (same results as IEEE division; tools/rcp_check.hip checks
// both over every float input on the GPU, log in profiles/).
#pragma once

// GIC_FASTDIV_HOST: div3_rn as a host function (tests/fastdiv_check.cpp); rcp_rn
// needs v_rcp_f32 and is device-only
#ifdef GIC_FASTDIV_HOST
#define GIC_FD inline
#else
#define GIC_FD __device__ __forceinline__
#endif

namespace gic {

// RN(d / 3): q0 = d * RN(1/3), r = d - 3 q0 exactly (FMA), q = q0 + r * RN(1/3);
// the sign of an exact zero follows d.  Equal to d / 3.0f for every finite d
// (tools/rcp_check.hip over all 2^32 inputs); a non-finite d is returned as it
// is -- inf / 3 = inf, and a NaN keeps its payload as the division would --
// where the sequence above would give NaN for +-inf.  The BC1 search divides
// such values only on unbounded float block inputs (huge or infinite texels
// through Image_CompressAMDBC1Block / GIC_SRC_FLOAT32).
GIC_FD float div3_rn(float d)
{
    const float C = 0x1.555556p-2f;
    const float q0 = d * C;
    const float r = __builtin_fmaf(-q0, 3.0f, d);
    const float q = __builtin_copysignf(__builtin_fmaf(r, C, q0), d);
    return __builtin_isfinite(d) ? q : d;
}

#ifndef GIC_FASTDIV_HOST
// RN(1 / s) for normal s away from the range ends: v_rcp_f32 (1 ulp) and one
// FMA Newton step; zero, denormal, huge and non-finite s take the IEEE sequence
__device__ __forceinline__ float rcp_rn(float s)
{
    const float a = __builtin_fabsf(s);
    if (!(a >= 0x1p-125f && a <= 0x1p125f)) return 1.0f / s;
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r0, 1.0f);
    return __builtin_fmaf(e, r0, r0);
}
#endif

}  // namespace gic
