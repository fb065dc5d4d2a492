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

// ---- the parallel header walk of large files --------------------------------
// read_next_header's chain is a linked list through the file (each header's
// ckSize gives the next one's offset): walked one header at a time it is a chain
// of dependent HBM reads (~1.4 us each, 1.4 ms for C2's 1,024 blocks).  Large
// files instead run
//   wv_dframe_scan   one workgroup per 8 KiB tile: every even offset (headers are
//                    2-B aligned: ckSize is even) tested against read_next_header's
//                    acceptance test, candidates kept in offset order;
//   wv_dframe_rank   one workgroup per file: the candidates' successors by binary
//                    search, list ranking by pointer jumping in LDS (the chain from
//                    offset 0 must end exactly at the file's end), each header's
//                    fields checked in parallel (block_index = prefix sum of the
//                    block_samples, total_samples = the sum).
// A candidate inside a payload that happens to pass the test either heads a chain
// that dies (ignored) or merges with the true chain and collides with a true
// block's rank: the file then falls back to the serial walk (ranked = 0).
// Candidates are stored compactly (each tile takes its range with one atomic
// add); the store is sized for one header per 32 bytes (a block is a 32-byte
// header plus its sub-blocks) and a file whose tiles overflow it is walked
// serially instead.
constexpr int kTile = 8192;
constexpr int kRankMax = 8192;           // candidates one workgroup ranks in LDS
constexpr uint32_t kNoRange = 0xFFFFFFFFu;

__device__ __forceinline__ bool hdr_ok(const uint8_t *b) {
    return b[0] == 'w' && b[1] == 'v' && b[2] == 'p' && b[3] == 'k' && (b[4] & 1) == 0 && b[6] < 16 && b[7] == 0 &&
           b[9] == 4 && b[8] >= (wvf::MIN_STREAM_VERS & 0xff) && b[8] <= (wvf::MAX_STREAM_VERS & 0xff);
}

// cnt[t]: tile t's candidates, cnt[ntiles + t]: their first index in `cand`
// (kNoRange: the store overflowed), cnt[2 ntiles]: the store's fill (zeroed first)
extern "C" __global__ void __launch_bounds__(256) wv_dframe_scan(const DFile *__restrict__ files,
                                                                 const uint32_t *__restrict__ tile_file,
                                                                 uint32_t ntiles,
                                                                 const uint8_t *__restrict__ blob,
                                                                 uint32_t *__restrict__ cand, uint32_t cand_cap,
                                                                 uint32_t *__restrict__ cnt) {
    __shared__ uint32_t buf[(kTile + 64) / 4];
    __shared__ uint32_t part[256];
    __shared__ uint32_t range0;
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    const DFile &F = files[tile_file[t]];
    const uint64_t start = (uint64_t)(t - F.tile0) * kTile;
    // the tile and 64 bytes past it (the blob is padded: files are 16-B aligned and the
    // last one is followed by 64 B of 0xFF), as dwords from a 16-B aligned base
    const uint32_t *src = reinterpret_cast<const uint32_t *>(blob + F.base + start);
    for (uint32_t i = tid; i < (kTile + 64) / 4; i += 256) buf[i] = start + 4 * (uint64_t)i < F.len + 32 ? src[i] : 0u;
    __syncthreads();
    const uint8_t *b = reinterpret_cast<const uint8_t *>(buf);
    // thread tid owns bytes [32 tid, 32 tid + 32) of the tile: 16 even offsets
    uint32_t mine = 0, found[16];
    for (int j = 0; j < 16; j++) {
        const uint32_t o = 32 * tid + 2 * j;
        const uint64_t p = start + o;
        if (p + 32 <= F.len && hdr_ok(b + o)) found[mine++] = (uint32_t)p;
    }
    part[tid] = mine;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {  // inclusive scan of the per-thread counts
        const uint32_t v = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    const uint32_t at = part[tid] - mine, total = part[255];
    if (tid == 255) {
        uint32_t r = total ? atomicAdd(&cnt[2 * ntiles], total) : 0u;
        if (total && r + total > cand_cap) r = kNoRange;
        range0 = r;
        cnt[t] = total;
        cnt[ntiles + t] = r;
    }
    __syncthreads();
    if (range0 != kNoRange)
        for (uint32_t j = 0; j < mine; j++) cand[range0 + at + j] = found[j];
}

extern "C" __global__ void __launch_bounds__(1024) wv_dframe_rank(DFile *__restrict__ files,
                                                                  const uint32_t *__restrict__ rank_files,
                                                                  uint32_t ntiles,
                                                                  const uint8_t *__restrict__ blob,
                                                                  const uint32_t *__restrict__ cand,
                                                                  const uint32_t *__restrict__ cnt,
                                                                  uint64_t *__restrict__ slots) {
    using namespace wvf;
    __shared__ uint32_t lds[4 * kRankMax];  // 128 KiB
    uint32_t *pos = lds;                               // candidates in offset order
    int32_t *nxt = reinterpret_cast<int32_t *>(lds + kRankMax);  // successor; -1 the file's end, -2 no header
    uint32_t *dist = lds + 2 * kRankMax;               // nodes from here to the chain's end
    uint32_t *aux = lds + 3 * kRankMax;                // hits per rank
    uint64_t *pre = reinterpret_cast<uint64_t *>(lds); // later (over pos and nxt): frames before block r
    uint64_t *tpart = reinterpret_cast<uint64_t *>(dist);  // later: per-thread partial sums
    __shared__ uint32_t tsum[1024];
    __shared__ int32_t verdict;
    __shared__ uint32_t ntot;
    const uint32_t tid = threadIdx.x;
    DFile &F = files[rank_files[blockIdx.x]];
    const uint8_t *f = blob + F.base;
    const uint64_t len = F.len;
    if (tid == 0) {
        verdict = 1;
        ntot = 0;
    }
    __syncthreads();
    for (uint32_t t = tid; t < F.ntiles; t += 1024)
        if (cnt[ntiles + F.tile0 + t] == kNoRange) verdict = 0;  // a tile overflowed the candidate store
    __syncthreads();
    if (verdict == 0) {
        if (tid == 0) F.ranked = 0;  // the serial walk
        return;
    }
    // gather the tiles' candidates in order (1,024 tiles per round)
    for (uint32_t t0 = 0; t0 < F.ntiles; t0 += 1024) {
        const uint32_t t = t0 + tid;
        const uint32_t c = t < F.ntiles ? cnt[F.tile0 + t] : 0u;
        tsum[tid] = c;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {
            const uint32_t v = tid >= d ? tsum[tid - d] : 0u;
            __syncthreads();
            tsum[tid] += v;
            __syncthreads();
        }
        const uint32_t base = ntot + tsum[tid] - c, tot = ntot + tsum[1023];
        if (tot <= kRankMax)
            for (uint32_t j = 0; j < c; j++) pos[base + j] = cand[cnt[ntiles + F.tile0 + t] + j];
        __syncthreads();
        if (tid == 0) ntot = tot;
        __syncthreads();
    }
    const uint32_t N = ntot;
    if (N > kRankMax || N == 0 || pos[0] != 0) {  // too many for LDS / no header at byte 0
        if (tid == 0) {
            F.ranked = (N > kRankMax) ? 0 : -1;
            F.why = DF_HEADER;
        }
        return;
    }
    // successors: the header after candidate j starts at pos + ckSize + 8
    for (uint32_t j = tid; j < N; j += 1024) {
        const uint8_t *b = f + pos[j];
        const uint64_t ck = (uint64_t)b[4] | ((uint64_t)b[5] << 8) | ((uint64_t)b[6] << 16) | ((uint64_t)b[7] << 24);
        const uint64_t nx = (uint64_t)pos[j] + ck + 8;
        int32_t s = -2;
        if (nx == len) {
            s = -1;
        } else if (nx < len) {
            uint32_t lo = j + 1, hi = N;  // successors lie ahead
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (pos[m] < nx) lo = m + 1;
                else hi = m;
            }
            if (lo < N && pos[lo] == nx) s = (int32_t)lo;
        }
        nxt[j] = s;
        dist[j] = 1;
    }
    __syncthreads();
    // pointer jumping: after ceil(log2 N) rounds every node points at its chain's end
    constexpr int kPer = kRankMax / 1024;
    for (uint32_t span = 1; span < N; span <<= 1) {
        int32_t nn[kPer];
        uint32_t nd[kPer];
        for (int q = 0; q < kPer; q++) {
            const uint32_t j = tid + 1024u * q;
            if (j < N) {
                const int32_t s = nxt[j];
                nn[q] = s >= 0 ? nxt[s] : s;
                nd[q] = s >= 0 ? dist[j] + dist[s] : dist[j];
            }
        }
        __syncthreads();
        for (int q = 0; q < kPer; q++) {
            const uint32_t j = tid + 1024u * q;
            if (j < N) {
                nxt[j] = nn[q];
                dist[j] = nd[q];
            }
        }
        __syncthreads();
    }
    const uint32_t n = dist[0];
    if (nxt[0] != -1 || n > len / 32 + 1) {  // the chain from byte 0 does not end at the file's end
        if (tid == 0) {
            F.ranked = -1;
            F.why = DF_WALK;
        }
        return;
    }
    // ranks: block r is the node n - r nodes before the end; a second node at a rank
    // is a false header merging into the chain (the serial walk settles the file)
    for (uint32_t r = tid; r < n; r += 1024) aux[r] = 0;
    __syncthreads();
    for (uint32_t j = tid; j < N; j += 1024)
        if (nxt[j] == -1 && dist[j] <= n) {
            const uint32_t r = n - dist[j];
            atomicAdd(&aux[r], 1u);
            slots[F.slot + r] = pos[j];  // rewritten by the serial walk if two nodes share a rank
        }
    __syncthreads();
    for (uint32_t r = tid; r < n; r += 1024)
        if (aux[r] != 1) verdict = 0;
    __syncthreads();
    if (verdict == 0) {
        if (tid == 0) F.ranked = 0;
        return;
    }
    // every header: the walk's conditions, block_samples into the prefix sums
    DHdr h0;
    dframe_header(f, len, 0, h0);
    int32_t bad = 0;
    uint64_t bs[kPer], part = 0;
    for (int q = 0; q < kPer; q++) {
        const uint32_t r = tid * kPer + q;  // thread tid owns ranks [8 tid, 8 tid + 8)
        bs[q] = 0;
        if (r < n) {
            DHdr h;
            dframe_header(f, len, slots[F.slot + r], h);
            const uint32_t fl = h.flags;
            if (h.block_samples == 0 || !(fl & INITIAL_BLOCK) || ((fl ^ h0.flags) & (DSD_FLAG | MONO_FLAG)) ||
                ((fl & FALSE_STEREO) && (fl & (MONO_FLAG | DSD_FLAG))))
                bad = DF_WALK;
            bs[q] = h.block_samples;
        }
        part += bs[q];
    }
    __syncthreads();  // pos, nxt, dist are free now
    tpart[tid] = part;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = tid >= d ? tpart[tid - d] : 0ull;
        __syncthreads();
        tpart[tid] += v;
        __syncthreads();
    }
    uint64_t run = tpart[tid] - part;  // frames before rank 8 tid
    for (int q = 0; q < kPer; q++) {
        const uint32_t r = tid * kPer + q;
        if (r < n) {
            pre[r] = run;
            run += bs[q];
        }
    }
    __syncthreads();
    for (int q = 0; q < kPer; q++) {
        const uint32_t r = tid * kPer + q;
        if (r < n) {
            DHdr h;
            dframe_header(f, len, slots[F.slot + r], h);
            if ((uint64_t)h.block_index != pre[r]) bad = DF_WALK;
        }
    }
    if (bad) atomicMax(&verdict, 2 + bad);
    __syncthreads();
    if (tid == 0) {
        const uint64_t total = tpart[1023];
        if (verdict > 1) {
            F.ranked = -1;
            F.why = (uint32_t)(verdict - 2);
        } else if (h0.total_samples == 0xFFFFFFFFLL || (uint64_t)h0.total_samples != total) {
            F.ranked = -1;
            F.why = DF_TOTAL;
        } else {
            F.ranked = 1;
            F.nblocks = n;
        }
    }
}

// cnt: 2 ntiles + 1 words; cand: cand_cap words
hipError_t launch_dframe_rank(DFile *files, const uint32_t *tile_file, uint32_t ntiles, const uint32_t *rank_files,
                              uint32_t nrank, const uint8_t *blob, uint32_t *cand, uint32_t cand_cap, uint32_t *cnt,
                              uint64_t *slots, hipStream_t s) {
    if (!nrank) return hipSuccess;
    hipError_t e = hipMemsetAsync(cnt + 2 * (size_t)ntiles, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(wv_dframe_scan, dim3(ntiles), dim3(256), 0, s, files, tile_file, ntiles, blob, cand, cand_cap,
                       cnt);
    hipLaunchKernelGGL(wv_dframe_rank, dim3(nrank), dim3(1024), 0, s, files, rank_files, ntiles, blob, cand, cnt,
                       slots);
    return hipGetLastError();
}

size_t dframe_tile_cap() { return kTile / 32; }  // candidate store per tile
size_t dframe_tile_bytes() { return kTile; }

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
