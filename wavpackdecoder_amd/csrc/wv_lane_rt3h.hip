// wv_lane_rt3h.hip -- the run-time list lane kernel for lists of 6..16 terms, hybrid (HYBRID_BITRATE) blocks
// (wv_lane.h lane_blocks_rt3: a parser and three reconstruction waves per 64 blocks).  Its
// own translation unit: it builds in parallel with the others.
#include <hip/hip_runtime.h>

#include "wv_lane.h"

namespace wvg {

__global__ void __launch_bounds__(lane::RT3_THREADS) wv_pcm_lane_rt3_hy(const BlockDesc *__restrict__ descs,
                                                                     const uint32_t *__restrict__ list, uint32_t n,
                                                                     const uint8_t *__restrict__ blob,
                                                                     int32_t *__restrict__ out,
                                                                     uint32_t *__restrict__ status,
                                                                     uint32_t *__restrict__ dbg) {
    lane::lane_blocks_rt3<1>(descs, list, n, blob, out, status, dbg);
}

hipError_t launch_lane_rt3_hy(dim3 gl, hipStream_t s, const BlockDesc *descs, const uint32_t *list, uint32_t n,
                              const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg) {
    hipLaunchKernelGGL(wv_pcm_lane_rt3_hy, gl, dim3(lane::RT3_THREADS), 0, s, descs, list, n, blob, out, status, dbg);
    return hipGetLastError();
}

}  // namespace wvg
