// wv_lane.hip -- the lane-per-block PCM kernels (wv_lane.h), one instantiation
// per term list (MONO: mono and false-stereo blocks; HY: 1 hybrid blocks, 2 hybrid blocks with
// their .wvc correction stream).  Their own translation
// unit: the lane kernels build in parallel with wv_decode.hip.
#include <hip/hip_runtime.h>

#include "wv_lane.h"

namespace wvg {

// (A/B builds: -DWV_LANE_WPE=1 tells the register allocator and scheduler that one
// wave per SIMD is all that runs -- the kernel's LDS already allows one workgroup per CU)
#ifndef WV_LANE_WPE
#define WV_LANE_WPE 0
#endif
#if WV_LANE_WPE
#define WV_LANE_ATTR __attribute__((amdgpu_waves_per_eu(1, 1)))
#else
#define WV_LANE_ATTR
#endif
template <bool MONO, int HY, int... Ts>
__global__ void __launch_bounds__(256) WV_LANE_ATTR wv_pcm_lane(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                  uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                  uint32_t *__restrict__ status, uint32_t *__restrict__ dbg) {
    lane::lane_blocks<MONO, HY, Ts...>(descs, list, n, blob, out, status, dbg);
}

// (wv_lane_rt.hip)
hipError_t launch_lane_rt(dim3 grid, dim3 block, hipStream_t s, const BlockDesc *descs, const uint32_t *list, uint32_t n,
                          const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg);

hipError_t launch_lane(int which, dim3 gl, dim3 bl, hipStream_t s, const BlockDesc *descs, const uint32_t *list,
                       uint32_t n, const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg) {
    switch (which) {
    case LANE_FAST: hipLaunchKernelGGL((wv_pcm_lane<false, 0, WVG_TS_FAST>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
#ifndef WV_LANE_ONLY_FAST  // (asm inspection builds: scripts/lane_asm.sh)
    case LANE_DEFAULT: hipLaunchKernelGGL((wv_pcm_lane<false, 0, WVG_TS_DEFAULT>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_M5: hipLaunchKernelGGL((wv_pcm_lane<true, 0, WVG_TS_M5>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_HIGH16: hipLaunchKernelGGL((wv_pcm_lane<false, 0, WVG_TS_HIGH16>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_MONO_HIGH16: hipLaunchKernelGGL((wv_pcm_lane<true, 0, WVG_TS_MONO_HIGH16>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_HY_DEFAULT: hipLaunchKernelGGL((wv_pcm_lane<false, 1, WVG_TS_DEFAULT>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_HY_WVC: hipLaunchKernelGGL((wv_pcm_lane<false, 2, WVG_TS_DEFAULT>), gl, bl, 0, s, descs, list, n, blob, out, status, dbg); break;
    case LANE_RT: return launch_lane_rt(gl, bl, s, descs, list, n, blob, out, status, dbg);
#endif
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace wvg
