// wv_dframe.hip -- device-side framing kernels over the
// shared code of wv_dframe.h.
//
//   wv_dframe_walk   one lane per file: WavpackOpenFileInput on the first block
//                    and the read_next_header chain (WavPackUtils.cs:36-120,
//                    600-671); a serial chain of dependent 32-B header reads,
//                    so the lanes of a wave walk different files
//   wv_dframe_block  one lane per block: the sub-block walk of unpack_init
//                    (UnpackUtils.cs:24-68, MetadataUtils.cs:15-192) and the
//                    block's descriptor + FileInfo contributions
//
// Both are latency-bound (a few dozen dependent byte reads per block, 1,408 B
// written per descriptor), run once per upload, and leave the decode kernels'
// inputs in HBM.
#include <hip/hip_runtime.h>

#include "wv_dframe.h"

namespace wvg {

extern "C" __global__ void __launch_bounds__(64) wv_dframe_walk(DFile *__restrict__ files, uint32_t n,
                                                                const uint8_t *__restrict__ blob,
                                                                uint64_t *__restrict__ slots) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DFile f = files[i];
    dframe_walk(f, blob, slots);
    files[i] = f;
}

// thread i frames block i of the device-framed range: blk_file[i] is its file,
// blk_k[i] its block number in that file
extern "C" __global__ void __launch_bounds__(64) wv_dframe_block(const DFile *__restrict__ files,
                                                                 const uint32_t *__restrict__ blk_file,
                                                                 const uint32_t *__restrict__ blk_k, uint32_t n,
                                                                 const uint8_t *__restrict__ blob,
                                                                 const uint64_t *__restrict__ slots,
                                                                 BlockDesc *__restrict__ descs,
                                                                 DBlock *__restrict__ recs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DFile f = files[blk_file[i]];
    BlockDesc d;
    DBlock r;
    dframe_block(f, blk_k[i], blob, slots, d, r);
    descs[i] = d;
    recs[i] = r;
}

hipError_t launch_dframe_walk(DFile *files, uint32_t n, const uint8_t *blob, uint64_t *slots, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(wv_dframe_walk, dim3((n + 63) / 64), dim3(64), 0, s, files, n, blob, slots);
    return hipGetLastError();
}

hipError_t launch_dframe_block(const DFile *files, const uint32_t *blk_file, const uint32_t *blk_k, uint32_t n,
                               const uint8_t *blob, const uint64_t *slots, BlockDesc *descs, DBlock *recs,
                               hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(wv_dframe_block, dim3((n + 63) / 64), dim3(64), 0, s, files, blk_file, blk_k, n, blob, slots,
                       descs, recs);
    return hipGetLastError();
}

}  // namespace wvg
