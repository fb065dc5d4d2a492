// wv_lane_rt.hip -- the lane-per-block PCM kernel for term lists read at run time
// (wv_lane.h: RChain, lane_blocks_rt): lossless blocks, mono or stereo, any list of up
// to 16 terms of -3..-1, 1..8, 17, 18 (UnpackUtils.cs:156-187) -- the lists without a
// compile-time instantiation (wv_lane.hip).  Its own translation unit: it builds in
// parallel with the others.
#include <hip/hip_runtime.h>

#include "wv_lane.h"

namespace wvg {

__global__ void __launch_bounds__(256) wv_pcm_lane_rt(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                      uint32_t n, const uint8_t *__restrict__ blob,
                                                      int32_t *__restrict__ out, uint32_t *__restrict__ status,
                                                      uint32_t *__restrict__ dbg) {
    lane::lane_blocks_rt(descs, list, n, blob, out, status, dbg);
}

// (wv_lane_rt3.hip: lists of 6..16 terms, lossless and hybrid kernels)
hipError_t launch_lane_rt3(dim3 gl, hipStream_t s, const BlockDesc *descs, const uint32_t *list, uint32_t n,
                           const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg);

hipError_t launch_lane_rt(dim3 gl, dim3 bl, hipStream_t s, const BlockDesc *descs, const uint32_t *list, uint32_t n,
                          const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg) {
    // (each pair of 64 list entries runs in the one kernel its first block's list length picks)
    hipLaunchKernelGGL(wv_pcm_lane_rt, gl, bl, 0, s, descs, list, n, blob, out, status, dbg);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
#if WV_RT_SPLIT16
    return launch_lane_rt3(gl, s, descs, list, n, blob, out, status, dbg);
#else
    return hipSuccess;
#endif
}

}  // namespace wvg
