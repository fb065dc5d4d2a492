// wv_decode.hip -- HIP kernels (gfx950) for the WavPack block decode.
//
// Kernel map:
//   wv_pcm_2wave<terms> : one workgroup (parser wave + reconstruction wave) per
//                         PCM block whose decorrelation term list is one of the
//                         shallow compile-time lists (fast, default, mono-5;
//                         wv_wave2.h).
//   wv_pcm_pipe<neg12>  : the same parser wave with the pipelined
//                         reconstruction wave (one pass per lane pair,
//                         wv_pipe.h) for every other term list (high, very
//                         high, 'extra', any list up to 16 terms).
//   wv_decode_pcm_wave  : one wave-uniform decode per PCM block whose fixup
//                         reads the int32 wvx stream; runs decode_pcm_block
//                         (get_words -> decorr passes -> joint/CRC/mute ->
//                         fixup -> int32 store) fused, sample-major.  Also one
//                         wave per chain of blocks that inherit decode state.
//   wv_decode_dsd_wave  : one wave-uniform decode per DSD block (DsdUtils modes
//                         0 and 3; stereo mode 3 with both channels' filters on
//                         the VALU).
//   wv_decode_dsd_fast  : mode 1, one wave per block with its tables in LDS.
//   wv_dsd_fill         : post-pass writing the 0x55 mute fills of DSD blocks in
//                         call-buffer coordinates (DsdUtils.cs:104-117, quirk B-9).
//   wv_meta_parse       : one lane per block finishing its descriptor with the
//                         deferred metadata values (wv_meta.h),
//                         once per upload, before any decode launch.
//   wv_format_pcm       : WavpackFormatSamples (WavPackUtils.cs:288-341) over the
//                         decoded batch, int32 -> little-endian PCM bytes.
// No MFMA: there is no contraction in this path; the work is serial integer
// bit-parsing per block, so the design goal is many independent blocks in
// flight with the whole per-sample pipeline in registers.
//
// Per-block aux word (aux[]): DSD blocks record the first muted chunk, PCM
// blocks the block frame of the residual whose decode raised the reference's
// C# exception (with ST_EXCEPTION).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "wv_decode_core.h"
#include "wv_meta.h"
#include "wv_wave2.h"
#include "wv_pipe.h"
#include "wv_lane.h"


namespace wvg {

// One 64-lane wave per block: every value derives from blockIdx.x, so the
// compiler keeps the decode wave-uniform (SGPRs, scalar branches, no
// divergence) and lane 0 alone stores.  Output value i of a block (frame * ints
// per frame + channel) goes to out[i]; the first `skip` values belong to a
// seek's discard calls and are dropped.
struct DevStoreWave {
    int32_t *out;
    uint64_t skip;
    bool lead;
    __device__ __forceinline__ void put(uint64_t i, int32_t v) {
        if (lead && i >= skip) out[i] = v;
    }
};

// A chain of blocks that inherit decode state (BlockDesc::inherit, B-8): the
// blocks in order, the PcmState of one handed to the next; a block that raises
// the reference's exception ends the chain (the reference stops there).
__device__ __noinline__ void decode_chain(const BlockDesc *__restrict__ descs, uint32_t head, const uint8_t *blob,
                                          int32_t *out, uint32_t *status, uint32_t *aux, PcmState &s) {
    const bool lead = threadIdx.x == 0;
    const uint32_t n = descs[head].chain_len;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t bi = head + k;
        const BlockDesc &d = descs[bi];
        DevStoreWave st{out + d.out_off, (uint64_t)d.pre_end * d.out_nch, lead};
        uint32_t exc = aux[bi];
        uint32_t r = d.fstatus | pcm_state_load(s, d, blob);
        r |= decode_pcm_run<DevStoreWave, true>(s, d, st, &exc);
        if (lead) {
            status[bi] = r;
            aux[bi] = exc;
        }
        if (r & ST_EXCEPTION) {
            // the members after it are never decoded (the reference stops here): their
            // status is the framing's, as the upload stored it (a poisoned status --
            // wvg_batch_poison's WVG_ST_UNWRITTEN -- must not survive the decode)
            if (lead)
                for (uint32_t j = k + 1; j < n; j++) status[head + j] = descs[head + j].fstatus;
            break;
        }
    }
}

extern "C" __global__ void __launch_bounds__(64) wv_decode_pcm_wave(const BlockDesc *__restrict__ descs,
                                                                    const uint32_t *__restrict__ list,
                                                                    const uint8_t *__restrict__ blob,
                                                                    int32_t *__restrict__ out,
                                                                    uint32_t *__restrict__ status,
                                                                    uint32_t *__restrict__ aux, uint32_t mode) {
    // the decode state in LDS: every lane of the (wave-uniform) decode reads and writes
    // the same values; in registers its run-time indexed pass rings went to scratch
    __shared__ PcmState ps;
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    // mode bit 2: only the blocks the .wvc lane kernel handed back (ST_REDO)
    if ((mode & 4u) && !(status[bi] & lane::ST_REDO)) return;
    if (d.chain_len >= 2) {
        decode_chain(descs, bi, blob, out, status, aux, ps);
        return;
    }
    const bool lead = threadIdx.x == 0;
    DevStoreWave st{out + d.out_off, (uint64_t)d.pre_end * d.out_nch, lead};
    uint32_t exc = (mode & 4u) ? 0u : aux[bi];
    const uint32_t s = d.fstatus | decode_pcm_block_in(ps, d, blob, st, &exc) | ((mode & 4u) ? (uint32_t)ST_REDONE : 0u);
    if (lead) {
        status[bi] = s;
        aux[bi] = exc;
    }
}

// hybrid stereo blocks of WavPack's default list with their .wvc stream (HYBRID_BITRATE,
// no HYBRID_BALANCE, not int32; no sticky state, seek or exact float): the .wvc lane
// kernel's candidates (wv_lane.h, HY == 2), the tail of the generic kernel's list
bool wvc_lane_candidate(const BlockDesc &d) {
    using namespace wvf;
    if (d.kind != KIND_PCM || !d.wvc_len || (d.flags & MONO_DATA) || d.out_nch != 2) return false;
    if ((d.flags & (HYBRID_FLAG | HYBRID_BITRATE | HYBRID_BALANCE | INT32_DATA)) != (HYBRID_FLAG | HYBRID_BITRATE))
        return false;
    if (d.chain_len >= 2 || d.inherit || d.xfloat || d.wvx_state || d.pre_end || d.fstatus) return false;
    static const int8_t def[5] = {WVG_TS_DEFAULT};
    if (d.num_terms != 5) return false;
    for (int i = 0; i < 5; i++)
        if (d.term[i] != def[i]) return false;
    return true;
}

// Mode 3's starting probability table for every rate_i (init_ptable,
// DsdUtils.cs:321-341; dsd_ptable_init), 256 KiB, filled once per device at
// wvg_open (upload_dsd_ptables): a block copies its row into LDS rather than
// running the up-to-3,469-step recurrence on its serial path (measured: 1.8 ms
// more per 22,050-frame block when each block built its own)
__device__ int32_t g_dsd_ptables[256 * 256];

// the table rows' device address (a kernel argument of the DSD lane kernel)
const int32_t *dsd_ptables_device() {
    static const int32_t *p = nullptr;
    if (!p) {
        void *a = nullptr;
        if (hipGetSymbolAddress(&a, HIP_SYMBOL(g_dsd_ptables)) == hipSuccess) p = (const int32_t *)a;
    }
    return p;
}
hipError_t launch_dsd3_lane(const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                            const int32_t *ptables, int32_t *out, uint32_t *status, uint32_t *mute_chunk,
                            uint32_t n_mono, hipStream_t s);

hipError_t launch_dsd1_lane(const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                            int32_t *out, uint32_t *status, uint32_t *mute_chunk, uint32_t n_mono, hipStream_t s);

hipError_t upload_dsd_ptables() {
    std::vector<int32_t> t(256 * 256);
    for (int r = 0; r < 256; r++) dsd_ptable_init(r, t.data() + (size_t)r * 256, 0, 1);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_dsd_ptables), t.data(), t.size() * sizeof(int32_t));
}

// Payload bytes for a wave-uniform decoder: aligned dwords through the scalar
// cache (one s_load per 4 bytes, the current dword kept in an SGPR) instead of
// a vector byte load, and its full memory latency, per byte.
struct ByteSrcWave {
    const uint32_t *w;  // the dword holding the payload's first byte
    uint32_t sh;        // the payload's first byte within it
    uint32_t cur_i, cur;
    // pointer arithmetic on the kernel argument (no integer round trip) keeps
    // the global address space, so the loads stay scalar, not flat
    __device__ __forceinline__ void init(const uint8_t *p) {
        sh = (uint32_t)((uintptr_t)p & 3);
        w = (const uint32_t *)(p - sh);
        cur_i = 0;
        cur = __builtin_amdgcn_readfirstlane(w[0]);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t bp) {
        const uint32_t a = bp + sh;
        if ((a >> 2) != cur_i) {
            cur_i = a >> 2;
            cur = __builtin_amdgcn_readfirstlane(w[cur_i]);
        }
        return (cur >> ((a & 3) * 8)) & 0xFFu;
    }
};

// Payload bytes for the DSD range coders: a 64-bit big-endian window of the
// next bytes (byte bp in bits 63..56), refilled a dword at a time from a
// dword loaded one refill ahead (a vector load, read into a scalar register
// at its refill, so the load latency is off the decode chain).  Reads run at most 12 bytes past the consumed position:
// inside the blob's 64-byte 0xFF tail at worst; bytes past the payload are
// never shifted in (callers cap n by the bytes left).
struct DsdWin {
    const uint32_t *w;
    uint64_t win;
    uint32_t avail;  // loaded bytes in win, >= 4 between calls
    uint32_t ni;     // index of the dword in nxt
    uint32_t nxt;
    static __device__ __forceinline__ uint32_t bswap_u(uint32_t x) {
        return (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)__builtin_bswap32(x));
    }
    __device__ __forceinline__ void init(const uint8_t *p) {
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
        w = (const uint32_t *)(p - sh);
        win = (uint64_t)bswap_u(w[0]) << (32u + 8u * sh);
        avail = 4u - sh;
        nxt = w[1];
        ni = 2;
        refill();
    }
    // nxt stays a vector register until the next refill moves it to a scalar
    // one: the load's wait lands there, ~4 payload bytes (tens of decisions) later
    __device__ __forceinline__ void refill() {  // avail <= 4
        win |= (uint64_t)bswap_u(nxt) << (32u - 8u * avail);
        avail += 4u;
        nxt = w[ni];
        ni++;
    }
    // v shifted left by n bytes (s = 8n, n <= 4) with the next n bytes below it
    __device__ __forceinline__ uint32_t shift_in(uint32_t v, uint32_t s, uint32_t n) {
        const uint64_t t = ((((uint64_t)v << 32) | (win >> 32)) << s) >> 32;
        win <<= s;
        avail -= n;
        if (avail < 4u) refill();
        return (uint32_t)t;
    }
};

// The DSD coders' renormalisation (DsdUtils.cs:295-300, 424-429) in one step:
// the byte loop shifts while the top bytes of high and low agree, and each
// shift moves high ^ low left by a byte (filling 0xFF), so it runs once per
// leading zero byte of high ^ low (4 when equal; none when the top bytes
// differ), capped by the payload bytes left.  Branch-free.
__device__ __forceinline__ void dsd_renorm(DsdWin &src, uint32_t &bp, uint32_t dlen, uint32_t &value, uint32_t &high,
                                           uint32_t &low) {
    uint32_t n = (uint32_t)__clz(high ^ low) >> 3;
    const uint32_t left = dlen - bp;
    n = n < left ? n : left;
    const uint32_t s = 8u * n;
    value = src.shift_in(value, s, n);
    high = (uint32_t)(((((uint64_t)high << 32) | 0xFFFFFFFFu) << s) >> 32);
    low = (uint32_t)((((uint64_t)low << 32) << s) >> 32);
    bp += n;
}

// Output of a wave-uniform DSD decoder staged in one vector register: value k
// of a run of up to 64 goes to lane k (a select), and the run is written by
// one 64-lane store.  A store per value from one lane would leave stores in
// flight at every payload refill, whose load wait (vmcnt) waits for them too.
struct StageOutWave {
    int32_t *out;
    uint64_t skip;  // values before this index are discarded (a seek's pre_end)
    uint64_t base;  // output index of lane 0
    uint32_t cnt;
    int32_t stg;
    __device__ __forceinline__ void flush() {
        const uint32_t lane = threadIdx.x;
        const uint64_t i = base + lane;
        if (lane < cnt && i >= skip) out[i] = stg;
        base += cnt;
        cnt = 0;
    }
    __device__ __forceinline__ void put1(int32_t v0) {
        const uint32_t lane = threadIdx.x;
        stg = lane == cnt ? v0 : stg;
        cnt += 1;
        if (cnt == 64) flush();
    }
    __device__ __forceinline__ void put2(int32_t v0, int32_t v1) {  // cnt stays even
        const uint32_t lane = threadIdx.x;
        stg = lane == cnt ? v0 : stg;
        stg = lane == cnt + 1 ? v1 : stg;
        cnt += 2;
        if (cnt == 64) flush();
    }
};

// DsdUtils.init_dsd_block_high + decode_high (DsdUtils.cs:343-493) for one
// block, wave-uniform, with the channel count a compile-time constant so the
// per-channel filter state (value, filter0..6, factor) lives in scalar
// registers.  Same results and status bits as decode_dsd_block's KIND_DSD_HIGH
// path (wv_decode_core.h), which the CPU tests check against the oracle.
template <int WCH>
__device__ __forceinline__ DsdResult dsd_high_wave(const BlockDesc &d, const uint8_t *blob, const uint8_t *tables,
                                                   int32_t *ptable, DevStoreWave &out) {
    using namespace wvf;
    const uint32_t flags = d.flags;
    const bool fstereo = (flags & FALSE_STEREO) != 0;
    const uint32_t och = (flags & MONO_FLAG) ? 1u : 2u;
    const uint32_t dlen = d.dsd_data_len;
    ByteSrcWave src;
    src.init(blob + d.bits_off);
    uint32_t bp = 0;
    int32_t crc = -1;
    DsdResult res = {0, 0};
    bool mute = false;
    uint32_t low = 0, high = 0xFFFFFFFFu, value = 0;
    for (int i = 0; i < 4; i++) value = (value << 8) | src.byte(bp++);
    {  // the block's initial probability table, 4 entries per lane
        const int32_t *pt0 = g_dsd_ptables + (uint32_t)(d.dsd_rate_i & 255) * 256u;
        for (uint32_t i = threadIdx.x; i < 256; i += 64) ptable[i] = pt0[i];
        __syncthreads();
    }
    int32_t q0[WCH], q1[WCH], q2[WCH], q3[WCH], q4[WCH], q5[WCH], q6[WCH], q7[WCH], q8[WCH], bytei[WCH];
#pragma unroll
    for (int c = 0; c < WCH; c++) {
        q0[c] = 0;
        q1[c] = 0;
        q2[c] = d.dsd_filters[c][0];
        q3[c] = d.dsd_filters[c][1];
        q4[c] = d.dsd_filters[c][2];
        q5[c] = d.dsd_filters[c][3];
        q6[c] = d.dsd_filters[c][4];
        q7[c] = 0;
        q8[c] = d.dsd_filters[c][5];
        bytei[c] = 0;
    }
    uint32_t f = 0, chunk_len = d.first_chunk, ci = 0;
    while (f < d.nframes) {
        uint32_t n = chunk_len;
        if (n > d.nframes - f) n = d.nframes - f;
        if (!mute) {
            for (uint32_t j = 0; j < n; j++) {
#pragma unroll
                for (int c = 0; c < WCH; c++) q0[c] = add32(sub32(q2[c], q6[c]), mul32(q7[c], q8[c]) >> 2);
                for (int bit = 0; bit < 8; bit++) {
#pragma unroll
                    for (int c = 0; c < WCH; c++) {
                        const int pp = (q0[c] >> 8) & 255;
                        const int32_t pv = __builtin_amdgcn_readfirstlane(ptable[pp]);
                        const uint32_t split = low + ((high - low) >> 8) * ((uint32_t)pv >> 16);
                        // branch-free: selects instead of a taken branch per decision
                        const bool zero = value <= split;
                        high = zero ? split : high;
                        low = zero ? low : split + 1;
                        ptable[pp] = pv + (((zero ? 0x010000FE : 0x00010000) - pv) >> 8);
                        q1[c] = zero ? -1 : 0;
                        while (((high ^ low) & 0xFF000000u) == 0 && bp < dlen) {
                            value = (value << 8) | src.byte(bp++);
                            high = (high << 8) | 0xFF;
                            low <<= 8;
                        }
                        q0[c] = add32(q0[c], mul32(q7[c], 8));
                        bytei[c] = shl32(bytei[c], 1) | (q1[c] & 1);
                        q8[c] = add32(q8[c], (((q0[c] ^ q1[c]) >> 31) | 1) & ((q0[c] ^ sub32(q0[c], mul32(q7[c], 16))) >> 31));
                        q2[c] = add32(q2[c], sub32(q1[c] & (1 << 20), q2[c]) >> 6);
                        q3[c] = add32(q3[c], sub32(q1[c] & (1 << 20), q3[c]) >> 4);
                        q4[c] = add32(q4[c], sub32(q3[c], q4[c]) >> 4);
                        q5[c] = add32(q5[c], sub32(q4[c], q5[c]) >> 4);
                        q0[c] = sub32(q5[c], q6[c]) >> 4;
                        q6[c] = add32(q6[c], q0[c]);
                        q7[c] = add32(q7[c], sub32(q0[c], q7[c]) >> 3);
                        q0[c] = add32(sub32(q2[c], q6[c]), mul32(q7[c], q8[c]) >> 2);
                    }
                }
                int32_t v[2] = {0, 0};
#pragma unroll
                for (int c = 0; c < WCH; c++) {
                    v[c] = bytei[c] & 0xFF;
                    q8[c] = sub32(q8[c], add32(q8[c], 512) >> 10);
                    crc = add32(crc, add32(shl32(crc, 1), v[c]));
                }
                const uint64_t o = (uint64_t)(f + j) * och;
                if (WCH == 1 && !fstereo) {
                    out.put(o, v[0]);
                } else if (fstereo) {
                    out.put(o, v[0]);
                    out.put(o + 1, v[0]);
                } else {
                    out.put(o, v[0]);
                    out.put(o + 1, v[1]);
                }
            }
            // DsdUtils.cs:99-101: the final chunk checks the crc and mutes on mismatch
            if (f + n == d.block_samples && crc != d.crc) mute = true;
        }
        if (mute && !(res.status & ST_DSD_MUTE)) {
            res.status |= ST_DSD_MUTE;
            res.mute_chunk = ci;
        }
        f += n;
        chunk_len = next_call_len(d, f);
        ci++;
    }
    if (d.nframes == d.block_samples) {
        res.status |= ST_CRC_CHECKED;
        if (crc != d.crc) res.status |= ST_CRC_ERROR;
    }
    return res;
}

// One range-coder decision of decode_high (DsdUtils.cs:409-422) on the scalar
// unit: split, compare, narrow; the outcome comes back as the lane mask M of
// the channel's lanes when the value is at or below the split (filter0 = -1),
// else 0.  In asm so the compare's SCC feeds all three selects.
template <uint32_t M>
__device__ __forceinline__ uint32_t dsd_decide(uint32_t value, uint32_t s, uint32_t &high, uint32_t &low) {
    uint32_t z, t, t1;
    asm("s_sub_u32 %[t], %[hi], %[lo]\n\t"
        "s_lshr_b32 %[t], %[t], 8\n\t"
        "s_mul_i32 %[t], %[t], %[s]\n\t"
        "s_add_u32 %[t], %[t], %[lo]\n\t"
        "s_add_u32 %[t1], %[t], 1\n\t"
        "s_cmp_le_u32 %[v], %[t]\n\t"
        "s_cselect_b32 %[hi], %[t], %[hi]\n\t"
        "s_cselect_b32 %[lo], %[lo], %[t1]\n\t"
        "s_cselect_b32 %[z], %[m], 0"
        : [hi] "+s"(high), [lo] "+s"(low), [z] "=s"(z), [t] "=&s"(t), [t1] "=&s"(t1)
        : [v] "s"(value), [s] "s"(s), [m] "i"(M)
        : "scc");
    return z;
}

// Stereo mode 3: lane 0 holds channel 0's filter state and lane 1 channel
// 1's (every even / odd lane a copy), so one VALU instruction updates both
// channels (the chains are independent; only the range coder and the ptable
// are shared).  A lone wave issues about one instruction per four cycles, so a
// decision costs what it issues plus whatever latency is left exposed.  Per bit
// (about 74 instructions for the two decisions):
//  * the LDS read of both channels' ptable entries is issued first, and the
//    factor step's decision-independent half (the sign test of value against
//    value - 16 filter6) is computed while it is in flight;
//  * the two decisions stay scalar and each returns its outcome as a lane mask
//    (even lanes channel 0's, odd lanes channel 1's), so filter0 is one select
//    and VALUE_ONE & filter0 one and;
//  * both channels' ptable updates are one per-lane LDS write (when both
//    channels hit one entry, channel 1's update starts from channel 0's and
//    channel 0's write goes to a spare slot, ptable[256]);
//  * filter6 and factor stay far inside 24 bits (|filter6| <= 2^16,
//    |factor| <= 2^15 + 8 for any stream: the filters are convex updates of
//    0 / 2^20 and the factor decays by 1/1024 per byte), so their products
//    are full-rate 24-bit multiplies with the same low 32 bits as C#'s
//    wrapping int multiply;
//  * each lane accumulates minus its channel's output byte as B = 2 B + filter0
//    (one shift-add), read out once per byte.
// Same results and status bits as dsd_high_wave<2> (DsdUtils.cs:391-493).
__device__ __forceinline__ DsdResult dsd_high_v2(const BlockDesc &d, const uint8_t *blob, const uint8_t *tables,
                                                 int32_t *ptable, DevStoreWave &out) {
    using namespace wvf;
    constexpr int32_t kUp = 0x010000FE, kDown = 0x00010000;
    const uint32_t dlen = d.dsd_data_len;
    const int ch = threadIdx.x & 1;
    DsdWin src;
    src.init(blob + d.bits_off);
    uint32_t bp = 0;
    int32_t crc = -1;
    DsdResult res = {0, 0};
    bool mute = false;
    uint32_t low = 0, high = 0xFFFFFFFFu, value = 0;
    value = src.shift_in(0, 32, 4);  // init_dsd_block_high checked >= 4 payload bytes
    bp = 4;
    {
        const int32_t *pt0 = g_dsd_ptables + (uint32_t)(d.dsd_rate_i & 255) * 256u;
        for (uint32_t i = threadIdx.x; i < 256; i += 64) ptable[i] = pt0[i];
        __syncthreads();
    }
    uint8_t *lds = (uint8_t *)ptable;
    StageOutWave so{out.out, out.skip, 0, 0, 0};
    int32_t q2 = d.dsd_filters[ch][0], q3 = d.dsd_filters[ch][1], q4 = d.dsd_filters[ch][2];
    int32_t q5 = d.dsd_filters[ch][3], q6 = d.dsd_filters[ch][4], q8 = d.dsd_filters[ch][5];
    int32_t q7 = 0;
    uint32_t f = 0, chunk_len = d.first_chunk, ci = 0;
    while (f < d.nframes) {
        uint32_t n = chunk_len;
        if (n > d.nframes - f) n = d.nframes - f;
        if (!mute) {
            for (uint32_t j = 0; j < n; j++) {
                int32_t q0 = add32(sub32(q2, q6), __mul24(q7, q8) >> 2);
                int32_t nb = 0;  // minus this lane's channel's output byte so far
#pragma unroll
                for (int bit = 0; bit < 8; bit++) {
                    const uint32_t addr = ((uint32_t)q0 >> 6) & 0x3FCu;
                    int32_t pv = *(const int32_t *)(lds + addr);
                    // decision-independent work, under the LDS latency
                    const int32_t v = add32(q0, shl32(q7, 3));
                    int32_t t;  // q0 - 8 * filter6, one 24-bit multiply-add
                    asm("v_mad_i32_i24 %0, %1, -8, %2" : "=v"(t) : "v"(q7), "v"(q0));
                    const int32_t sx = (v ^ t) >> 31;
                    const uint32_t pa0 = (uint32_t)__builtin_amdgcn_readlane((int32_t)addr, 0);
                    const uint32_t pa1 = (uint32_t)__builtin_amdgcn_readlane((int32_t)addr, 1);
                    const bool alias = pa0 == pa1;
                    // computed before the first use of pv, i.e. while the read is in flight
                    asm volatile("" : "+v"(pv) : "v"(sx), "s"(pa0), "s"(pa1));
                    // channel 0's decision
                    const uint32_t ps = (uint32_t)pv >> 16;
                    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int32_t)ps, 0);
                    uint32_t s1 = (uint32_t)__builtin_amdgcn_readlane((int32_t)ps, 1);
                    const uint32_t z0 = dsd_decide<0x55555555u>(value, s0, high, low);
                    int32_t pvl = pv;
                    uint32_t wa = addr;
                    if (__builtin_expect(alias, 0)) {  // channel 1 reads channel 0's updated entry
                        const int32_t p0 = __builtin_amdgcn_readlane(pv, 0);
                        const int32_t np0 = p0 + (((z0 ? kUp : kDown) - p0) >> 8);
                        s1 = (uint32_t)np0 >> 16;
                        pvl = ch ? np0 : pv;
                        wa = ch ? addr : 1024u;
                    }
                    if (__builtin_expect((high ^ low) < 0x1000000u, 0)) dsd_renorm(src, bp, dlen, value, high, low);
                    // channel 1's decision
                    const uint32_t z1 = dsd_decide<0xAAAAAAAAu>(value, s1, high, low);
                    if (__builtin_expect((high ^ low) < 0x1000000u, 0)) dsd_renorm(src, bp, dlen, value, high, low);
                    // this lane's channel's filter0: even lanes take z0, odd lanes z1
                    const uint32_t zlo = z0 | z1;
                    const bool zl = __builtin_amdgcn_inverse_ballot_w64(((uint64_t)zlo << 32) | zlo);
                    const int32_t f0 = zl ? -1 : 0;
                    nb = add32(shl32(nb, 1), f0);
                    *(int32_t *)(lds + wa) = pvl + (((zl ? kUp : kDown) - pvl) >> 8);
                    q8 = add32(q8, sx & (((v ^ f0) >> 31) | 1));
                    const int32_t x = f0 & (1 << 20);
                    q2 = add32(q2, sub32(x, q2) >> 6);
                    q3 = add32(q3, sub32(x, q3) >> 4);
                    q4 = add32(q4, sub32(q3, q4) >> 4);
                    q5 = add32(q5, sub32(q4, q5) >> 4);
                    const int32_t dd = sub32(q5, q6) >> 4;
                    q6 = add32(q6, dd);
                    q7 = add32(q7, sub32(dd, q7) >> 3);
                    q0 = add32(sub32(q2, q6), __mul24(q7, q8) >> 2);
                }
                const int32_t v0 = -__builtin_amdgcn_readlane(nb, 0), v1 = -__builtin_amdgcn_readlane(nb, 1);
                q8 = sub32(q8, add32(q8, 512) >> 10);
                crc = add32(crc, add32(shl32(crc, 1), v0));
                crc = add32(crc, add32(shl32(crc, 1), v1));
                so.put2(v0, v1);
            }
            so.flush();
            if (f + n == d.block_samples && crc != d.crc) mute = true;
        }
        if (mute && !(res.status & ST_DSD_MUTE)) {
            res.status |= ST_DSD_MUTE;
            res.mute_chunk = ci;
        }
        f += n;
        so.base = (uint64_t)f * 2u;
        chunk_len = next_call_len(d, f);
        ci++;
    }
    if (d.nframes == d.block_samples) {
        res.status |= ST_CRC_CHECKED;
        if (crc != d.crc) res.status |= ST_CRC_ERROR;
    }
    return res;
}

// DsdUtils mode 1's tables (prob u8, summed u16, lookup u8, value_lookup i32;
// 16-B aligned by the framing) read through the scalar cache: a data-dependent
// table read costs a scalar-cache hit, not a vector load's memory latency
struct DsdTablesWave {
    w2::cdw_ptr t;
    int bins;
    __device__ __forceinline__ uint32_t u8(uint32_t i) const { return (t[i >> 2] >> ((i & 3) * 8)) & 0xFFu; }
    __device__ __forceinline__ uint32_t prob(uint32_t i) const { return u8(i); }
    __device__ __forceinline__ uint32_t summed(uint32_t i) const {
        const uint32_t b = (uint32_t)bins * 256u + 2u * i;
        return (t[b >> 2] >> ((b & 2) * 8)) & 0xFFFFu;
    }
    __device__ __forceinline__ uint32_t lookup(uint32_t i) const { return u8((uint32_t)bins * 768u + i); }
    __device__ __forceinline__ int32_t vlook(uint32_t i) const { return (int32_t)t[(uint32_t)bins * 512u + i]; }
};

// DsdUtils modes 0 (raw bytes) and 1 (init_dsd_block_fast + decode_fast,
// DsdUtils.cs:149-304), wave-uniform, channel count a template parameter.
// Same results and status bits as decode_dsd_block (wv_decode_core.h).
template <int WCH, bool FAST>
__device__ __forceinline__ DsdResult dsd_simple_wave(const BlockDesc &d, const uint8_t *blob, const uint8_t *tables,
                                                     DevStoreWave &out) {
    using namespace wvf;
    const bool fstereo = (d.flags & FALSE_STEREO) != 0;
    const uint32_t och = (d.flags & MONO_FLAG) ? 1u : 2u;
    const uint32_t dlen = d.dsd_data_len;
    ByteSrcWave src;
    src.init(blob + d.bits_off);
    DsdTablesWave tb;
    tb.t = (w2::cdw_ptr)(tables + d.dsd_table_off);
    tb.bins = d.dsd_history_bins;
    const uint32_t bmask = (uint32_t)d.dsd_history_bins - 1u;
    uint32_t bp = 0;
    int32_t crc = -1;
    DsdResult res = {0, 0};
    bool mute = false;
    uint32_t low = 0, high = 0xFFFFFFFFu, value = 0;
    uint32_t p0 = 0, p1 = 0;
    if (FAST)
        for (int i = 0; i < 4; i++) value = (value << 8) | src.byte(bp++);
    uint32_t f = 0, chunk_len = d.first_chunk, ci = 0;
    while (f < d.nframes) {
        uint32_t n = chunk_len;
        if (n > d.nframes - f) n = d.nframes - f;
        bool chunk_ok = true;
        if (!mute) {
            for (uint32_t j = 0; j < n && chunk_ok; j++) {
                int32_t v[2] = {0, 0};
#pragma unroll
                for (int c = 0; c < WCH; c++) {
                    uint32_t code;
                    if (!FAST) {
                        code = bp < dlen ? src.byte(bp) : 0u;
                        bp++;
                    } else {
                        const uint32_t pi = p0 * 256u;
                        const uint32_t tot = tb.summed(pi + 255u);
                        if (tot == 0) { chunk_ok = false; break; }
                        uint32_t mult = (high - low) / tot;
                        if (mult == 0) {
                            if (dlen - bp >= 4)
                                for (int i = 0; i < 4; i++) value = (value << 8) | src.byte(bp++);
                            low = 0;
                            high = 0xFFFFFFFFu;
                            mult = high / tot;
                            if (mult == 0) { chunk_ok = false; break; }
                        }
                        const uint32_t index = (value - low) / mult;
                        if (index >= tot) { chunk_ok = false; break; }
                        code = tb.lookup((uint32_t)tb.vlook(p0) + index);
                        if (code > 0) low += tb.summed(pi + code - 1u) * mult;
                        high = low + tb.prob(pi + code) * mult - 1u;
                        if (WCH == 1) {
                            p0 = code & bmask;
                        } else {
                            p0 = p1;
                            p1 = code & bmask;
                        }
                        while (((high ^ low) & 0xFF000000u) == 0 && bp < dlen) {
                            value = (value << 8) | src.byte(bp++);
                            high = (high << 8) | 0xFF;
                            low <<= 8;
                        }
                    }
                    v[c] = (int32_t)code;
                }
                if (!chunk_ok) break;
#pragma unroll
                for (int c = 0; c < WCH; c++) crc = add32(crc, add32(shl32(crc, 1), v[c]));
                const uint64_t o = (uint64_t)(f + j) * och;
                if (WCH == 1 && !fstereo) {
                    out.put(o, v[0]);
                } else if (fstereo) {
                    out.put(o, v[0]);
                    out.put(o + 1, v[0]);
                } else {
                    out.put(o, v[0]);
                    out.put(o + 1, v[1]);
                }
            }
            if (!chunk_ok) {
                mute = true;
                res.status |= ST_NONDET;  // the rest of this chunk's region keeps stale caller data
            }
            // DsdUtils.cs:99-101: the final chunk checks the crc and mutes on mismatch
            if (!mute && f + n == d.block_samples && crc != d.crc) mute = true;
        }
        if (mute && !(res.status & ST_DSD_MUTE)) {
            res.status |= ST_DSD_MUTE;
            res.mute_chunk = ci;
        }
        f += n;
        chunk_len = next_call_len(d, f);
        ci++;
    }
    if (d.nframes == d.block_samples) {
        res.status |= ST_CRC_CHECKED;
        if (crc != d.crc) res.status |= ST_CRC_ERROR;
    }
    return res;
}

// DsdUtils mode 0 (DsdUtils.cs:73-82): the payload bytes ARE the output
// values, in order, and crc = 3 crc + v over them -- lane-parallel instead of a
// serial byte loop.  Value i (of N = nframes x channels read) is handled by
// lane i % 64, kDsdRawU values per lane per step (one byte load each, all in
// flight together; each load and each store instruction covers 64 consecutive
// values).  The CRC is a power-of-3 weighted sum: lane l keeps
// acc_l = sum_j v(l + 64 j) 3^(64 (J-1-j)) by Horner (acc = acc 3^64 + v), so
// with the values padded by zeros to Npad = 64 J
//   sum_i 3^(Npad-1-i) v_i = sum_l 3^(63-l) acc_l,
// the padding multiplies the true sum by 3^(Npad-N) (undone with 3's inverse
// mod 2^32), and crc = 3^N (-1) + sum.  Same outputs, status bits and mute
// chunk as dsd_simple_wave<WCH, false>: the only mute of mode 0 is the final
// chunk's CRC test (DsdUtils.cs:99-101); wv_dsd_fill writes its 0x55.
constexpr uint32_t kDsdRawU = 16;
template <int WCH>
__device__ __forceinline__ DsdResult dsd_raw_lanes(const BlockDesc &d, const uint8_t *blob, int32_t *out) {
    const bool fstereo = (d.flags & wvf::FALSE_STEREO) != 0;
    const uint32_t N = d.nframes * (uint32_t)WCH;  // values read (one byte each)
    const uint32_t dlen = d.dsd_data_len;          // (init_dsd_block: == block_samples x channels)
    const uint64_t skip = (uint64_t)d.pre_end * d.out_nch;  // a seek's discarded values
    const uint8_t *src = blob + d.bits_off;
    const uint32_t lane = threadIdx.x;
    constexpr uint32_t C64 = 0x797EBD01u;  // 3^64 mod 2^32
    uint32_t acc = 0;
    const uint32_t steps = (N + 64u * kDsdRawU - 1u) / (64u * kDsdRawU);
    for (uint32_t st = 0; st < steps; st++) {
        const uint32_t base = st * 64u * kDsdRawU + lane;
        uint32_t v[kDsdRawU];
#pragma unroll
        for (uint32_t u = 0; u < kDsdRawU; u++) {
            const uint32_t i = base + 64u * u;
            v[u] = (i < N && i < dlen) ? (uint32_t)src[i] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kDsdRawU; u++) {
            const uint32_t i = base + 64u * u;
            acc = acc * C64 + v[u];
            if (i < N) {
                if (!fstereo) {
                    if (i >= skip) out[i] = (int32_t)v[u];
                } else {
                    const uint64_t o = 2ull * i;
                    if (o >= skip) out[o] = (int32_t)v[u];
                    if (o + 1 >= skip) out[o + 1] = (int32_t)v[u];
                }
            }
        }
    }
    uint32_t part = acc * w2::upow_u32(3u, 63u - lane);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) part += (uint32_t)__shfl_xor((int)part, o);
    const uint32_t npad = steps * 64u * kDsdRawU;
    const uint32_t sum = part * w2::upow_u32(0xAAAAAAABu, npad - N);  // 3 * 0xAAAAAAAB == 1 mod 2^32
    const int32_t crc = (int32_t)(sum - w2::upow_u32(3u, N));
    DsdResult res = {0, 0};
    if (d.nframes == d.block_samples) {
        res.status |= ST_CRC_CHECKED;
        if (crc != d.crc) {
            res.status |= ST_CRC_ERROR;
            if (d.nframes) {  // the final call mutes: its index in the call schedule
                uint32_t f = 0, n = d.first_chunk, ci = 0;
                while (n && f + (n < d.nframes - f ? n : d.nframes - f) < d.nframes) {
                    f += n;
                    n = next_call_len(d, f);
                    ci++;
                }
                res.status |= ST_DSD_MUTE;
                res.mute_chunk = ci;
            }
        }
    }
    return res;
}

// A chain of DSD blocks continuing each other's DSD state (Appendix B-8 for DSD:
// a block without ID_DSD_BLOCK, or read without unpack_init): the blocks in order,
// the DsdState of one handed to the next (decode_dsd_chained, wv_decode_core.h);
// each block's status and first muted chunk are its own (wv_dsd_fill reads them)
__device__ __noinline__ void decode_dsd_chain(const BlockDesc *__restrict__ descs, uint32_t head,
                                              const uint8_t *blob, const uint8_t *tables, int32_t *ptable,
                                              int32_t *out, uint32_t *status, uint32_t *mute_chunk, uint32_t mode) {
    const bool lead = threadIdx.x == 0;
    const uint32_t n = descs[head].chain_len;
    DsdState S;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t bi = head + k;
        const BlockDesc &d = descs[bi];
        DevStoreWave st{out + d.out_off, (uint64_t)d.pre_end * d.out_nch, lead};
        const DsdResult r = decode_dsd_chained(S, d, k == 0, blob, tables, ptable, st, g_dsd_ptables);
        if (lead) {
            status[bi] = d.fstatus | r.status | ((k == 0 && (mode & 4u)) ? (uint32_t)ST_REDONE : 0u);
            mute_chunk[bi] = r.mute_chunk;
        }
    }
}

extern "C" __global__ void __launch_bounds__(64) wv_decode_dsd_wave(const BlockDesc *__restrict__ descs,
                                                                    const uint32_t *__restrict__ list,
                                                                    const uint8_t *__restrict__ blob,
                                                                    const uint8_t *__restrict__ tables,
                                                                    int32_t *__restrict__ out,
                                                                    uint32_t *__restrict__ status,
                                                                    uint32_t *__restrict__ mute_chunk,
                                                                    uint32_t mode) {
    __shared__ int32_t pt_lds[260];  // mode 3's adaptive ptable, one per block (+ dsd_high_v2's spare slot)
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    // mode bit 0: skip mode-1 blocks (wv_decode_dsd_fast's); bit 1: skip mode-3 blocks
    // (the lane kernel's, wv_dsd_lane.hip); bit 2: only the blocks the lane kernel
    // handed back (ST_REDO)
    if ((mode & 1u) && d.kind == KIND_DSD_FAST) return;
    if ((mode & 2u) && d.kind == KIND_DSD_HIGH) return;
    if ((mode & 4u) && !(status[bi] & lane::ST_REDO)) return;
    if (d.inherit & INH_MEMBER) return;  // decoded by its chain's first block
    if (d.chain_len >= 2) {
        decode_dsd_chain(descs, bi, blob, tables, pt_lds, out, status, mute_chunk, mode);
        return;
    }
    const bool lead = threadIdx.x == 0;
    DevStoreWave st{out + d.out_off, (uint64_t)d.pre_end * d.out_nch, lead};
    DsdResult r;
    // a mode-3 block is the batch's longest serial chain: its wave wins the
    // issue arbitration against the PCM waves sharing its SIMD
    if (d.kind == KIND_DSD_HIGH) __builtin_amdgcn_s_setprio(3);
    if (d.kind == KIND_DSD_HIGH)
        r = (d.flags & wvf::MONO_DATA) ? dsd_high_wave<1>(d, blob, tables, pt_lds, st)
                                       : dsd_high_v2(d, blob, tables, pt_lds, st);
    else if (d.kind == KIND_DSD_FAST)
        r = (d.flags & wvf::MONO_DATA) ? dsd_simple_wave<1, true>(d, blob, tables, st)
                                       : dsd_simple_wave<2, true>(d, blob, tables, st);
    else if (d.kind == KIND_DSD_RAW)
        r = (d.flags & wvf::MONO_DATA) ? dsd_raw_lanes<1>(d, blob, out + d.out_off)
                                       : dsd_raw_lanes<2>(d, blob, out + d.out_off);
    else
        r = decode_dsd_block(d, blob, tables, pt_lds, st, g_dsd_ptables);
    if (lead) {
        status[bi] = d.fstatus | r.status | ((mode & 4u) ? (uint32_t)ST_REDONE : 0u);
        mute_chunk[bi] = r.mute_chunk;
    }
}

// DsdUtils mode 1 (decode_fast, DsdUtils.cs:244-304) without its two 32-bit
// divisions per symbol.  The block's cumulative table (summed_probabilities,
// widened to u32) sits in LDS, one 1-KiB row per history bin; lane L holds the
// current bin's entries 4L..4L+3.  Per symbol:
//  * mult = (high - low) / tot by an invariant-divisor reciprocal
//    (Granlund-Montgomery: one mul_hi, four shifts/adds) whose constants lane b
//    holds for bin b and the wave reads with v_readlane;
//  * the decoded code is lookup[value_lookup[p0] + (value - low) / mult], i.e.
//    the number of entries with summed[i] <= (value - low) / mult, i.e. with
//    summed[i] * mult <= value - low (no product overflows: summed[i] <= tot
//    and tot * mult <= high - low): four products and compares per lane and a
//    popcount of the four ballots.  All 256 true <=> index >= tot (the C#
//    `return 0`);
//  * low and high move by summed[code - 1] * mult and summed[code] * mult, the
//    products themselves, picked in the lane that holds entry `code` (entry
//    code - 1 may be the previous lane's last one: a wave shift).
// Stereo reads the next symbol's row (p1) a symbol ahead.  Same results and
// status bits as dsd_simple_wave<WCH, true> (DsdUtils.cs:149-304).
template <int WCH>
__device__ __forceinline__ DsdResult dsd_fast_v2(const BlockDesc &d, const uint8_t *blob, const uint32_t *rows,
                                                 uint32_t vmag, uint32_t vsh1, uint32_t vsh2,
                                                 DevStoreWave &out) {
    using namespace wvf;
    const bool fstereo = (d.flags & FALSE_STEREO) != 0;
    const uint32_t och = (d.flags & MONO_FLAG) ? 1u : 2u;
    const uint32_t dlen = d.dsd_data_len;
    const uint32_t lane = threadIdx.x;
    DsdWin src;
    src.init(blob + d.bits_off);
    const uint32_t bmask = (uint32_t)d.dsd_history_bins - 1u;
    uint32_t bp = 0;
    int32_t crc = -1;
    DsdResult res = {0, 0};
    bool mute = false;
    uint32_t low = 0, high = 0xFFFFFFFFu, value = 0;
    uint32_t p0 = 0, p1 = 0;
    value = src.shift_in(0, 32, 4);  // init_dsd_block_fast checked >= 4 payload bytes
    bp = 4;
    uint4 row = *(const uint4 *)(rows + lane * 4u);  // bin 0
    StageOutWave so{out.out, out.skip, 0, 0, 0};
    uint32_t f = 0, chunk_len = d.first_chunk, ci = 0;
    while (f < d.nframes) {
        uint32_t n = chunk_len;
        if (n > d.nframes - f) n = d.nframes - f;
        bool chunk_ok = true;
        if (!mute) {
            for (uint32_t j = 0; j < n && chunk_ok; j++) {
                int32_t v[2] = {0, 0};
#pragma unroll
                for (int c = 0; c < WCH; c++) {
                    // the next symbol's row, while this one decodes (stereo: its bin is known)
                    uint4 nrow;
                    if (WCH == 2) nrow = *(const uint4 *)(rows + p1 * 256u + lane * 4u);
                    // (a bin with no counts, the C#'s first `return 0`, has an all-zero row: every
                    // product below is <= value - low, so code = 256 fails it; mult is then
                    // range (zero constants) and a mult == 0 reload before that changes nothing
                    // the failed chunk leaves behind)
                    const uint32_t mag = (uint32_t)__builtin_amdgcn_readlane((int32_t)vmag, (int32_t)p0);
                    const uint32_t s1 = (uint32_t)__builtin_amdgcn_readlane((int32_t)vsh1, (int32_t)p0);
                    const uint32_t s2 = (uint32_t)__builtin_amdgcn_readlane((int32_t)vsh2, (int32_t)p0);
                    uint32_t range = high - low;
                    uint32_t t1 = __umulhi(mag, range);
                    uint32_t mult = (t1 + ((range - t1) >> s1)) >> s2;
                    if (__builtin_expect(mult == 0, 0)) {
                        if (dlen - bp >= 4) {
                            value = src.shift_in(value, 32, 4);
                            bp += 4;
                        }
                        low = 0;
                        high = 0xFFFFFFFFu;
                        t1 = __umulhi(mag, high);
                        mult = (t1 + ((high - t1) >> s1)) >> s2;
                        if (mult == 0) { chunk_ok = false; break; }
                    }
                    const uint32_t x = value - low;
                    const uint32_t q0 = row.x * mult, q1 = row.y * mult, q2 = row.z * mult, q3 = row.w * mult;
                    const bool c0 = q0 <= x, c1 = q1 <= x, c2 = q2 <= x, c3 = q3 <= x;
                    const uint32_t code = (uint32_t)(__popcll(__ballot(c0)) + __popcll(__ballot(c1)) +
                                                     __popcll(__ballot(c2)) + __popcll(__ballot(c3)));
                    if (code >= 256u) { chunk_ok = false; break; }  // index >= tot
                    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)q3, 0x138, 0xf, 0xf, true);
                    const uint32_t hi_l = c0 ? (c1 ? (c2 ? q3 : q2) : q1) : q0;
                    const uint32_t lo_l = c3 ? q3 : (c2 ? q2 : (c1 ? q1 : (c0 ? q0 : prev)));
                    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int32_t)hi_l, (int32_t)(code >> 2));
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int32_t)lo_l, (int32_t)(code >> 2));
                    high = low + hi - 1u;
                    low = low + lo;
                    if (WCH == 1) {
                        p0 = code & bmask;
                        row = *(const uint4 *)(rows + p0 * 256u + lane * 4u);
                    } else {
                        p0 = p1;
                        p1 = code & bmask;
                        row = nrow;
                    }
                    dsd_renorm(src, bp, dlen, value, high, low);  // branch-free: ~a byte per symbol
                    v[c] = (int32_t)code;
                }
                if (!chunk_ok) break;
#pragma unroll
                for (int c = 0; c < WCH; c++) crc = add32(crc, add32(shl32(crc, 1), v[c]));
                if (WCH == 1 && !fstereo)
                    so.put1(v[0]);
                else if (fstereo)
                    so.put2(v[0], v[0]);
                else
                    so.put2(v[0], v[1]);
            }
            so.flush();
            if (!chunk_ok) {
                mute = true;
                res.status |= ST_NONDET;  // the rest of this chunk's region keeps stale caller data
            }
            if (!mute && f + n == d.block_samples && crc != d.crc) mute = true;
        }
        if (mute && !(res.status & ST_DSD_MUTE)) {
            res.status |= ST_DSD_MUTE;
            res.mute_chunk = ci;
        }
        f += n;
        so.base = (uint64_t)f * och;
        chunk_len = next_call_len(d, f);
        ci++;
    }
    if (d.nframes == d.block_samples) {
        res.status |= ST_CRC_CHECKED;
        if (crc != d.crc) res.status |= ST_CRC_ERROR;
    }
    return res;
}

// inclusive prefix sum over the wave's 64 lanes
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = (int)threadIdx.x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    return x;
}

// init_dsd_block_fast's tables (DsdUtils.cs:169-229) in LDS, from the block's
// probability data: the probabilities (run-length coded unless max_probability
// is 0xFF: a code above max_probability is a run of code - max_probability
// zeros, a code 1..max_probability one probability, 0 the end) into tab[bin *
// 256 + i], then each bin's running sums (summed_probabilities, ushort) in place.
// The framing ran the reference's checks on the same bytes (the data fills
// exactly bins x 256 entries, the totals are in range), so the wave decodes 64
// codes per step: a prefix sum of their run lengths gives each value its entry.
// Codes read past the terminating one (at most 63 bytes) stay inside the blob
// (the value bytes and the payload follow).
#ifndef WV_M1_HOSTTAB
#define WV_M1_HOSTTAB 0
#endif
//
// Everything happens inside the 32-KiB row region (no LDS beyond it, so as many
// waves per CU as the rows alone allow): the probabilities go to a byte array at
// bytes [0, 8 KiB), the staged data sits at [8 KiB, 16.25 KiB), and the rows are
// written last bin first -- row b covers the bytes of bins 4b .. 4b + 3, all
// already summed by then (bin 0's own bytes are read before its row is written).
constexpr uint32_t kDsdProbStage = 8192u + 256u;  // bytes: up to 32 x 256 codes + the end codes + over-read
constexpr uint32_t kDsdStageAt = 2048u;            // dwords: the stage follows the 8-KiB byte array
__device__ __forceinline__ void dsd_fast_tables(const BlockDesc &d, const uint8_t *blob, uint32_t bins, uint32_t *tab) {
    const uint32_t lane = threadIdx.x;
    const uint32_t ne = bins * 256u;
    uint8_t *pb = (uint8_t *)tab;
    uint32_t *stg = tab + kDsdStageAt;
    // the probability data (up to the 4 value bytes at bits_off) staged in LDS with
    // dword loads, all in flight together, instead of a byte load per code step
    const uint64_t a0 = d.dsd_prob_off & ~(uint64_t)3;
    const uint32_t sh = (uint32_t)(d.dsd_prob_off & 3);
    const uint64_t nb = d.bits_off > d.dsd_prob_off ? d.bits_off - d.dsd_prob_off : 0;
    const bool staged = nb + sh + 64u + 4u <= kDsdProbStage;
    if (staged) {
        const uint32_t nd = (uint32_t)((sh + nb + 64u + 3u) / 4u);  // + the codes read past the end
        const uint32_t *g = (const uint32_t *)(blob + a0);
#pragma unroll 8
        for (uint32_t i = lane; i < nd; i += 64) stg[i] = g[i];
        __syncthreads();
    }
    auto byte_at = [&](uint32_t k) -> uint32_t {
        if (!staged) return blob[d.dsd_prob_off + k];
        const uint32_t q = sh + k;
        return (stg[q >> 2] >> ((q & 3u) * 8u)) & 0xFFu;
    };
    if (d.dsd_max_prob < 0xFF) {
        const uint32_t maxp = (uint32_t)d.dsd_max_prob;
        for (uint32_t i = lane; i < ne / 16u; i += 64) ((uint4 *)pb)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        uint32_t outptr = 0, p = 0;
        while (outptr < ne) {
            const uint32_t c = byte_at(p + lane);
            const uint32_t len = c > maxp ? c - maxp : (c != 0 ? 1u : 0u);
            const uint32_t incl = wave_incl_scan(len);
            // the loop ends at the first 0 code, or once the entries are all filled
            const uint64_t ev = __ballot(c == 0 || outptr + incl >= ne);
            const uint32_t last = ev ? (uint32_t)__builtin_ctzll(ev) : 63u;
            if (lane <= last && c != 0 && c <= maxp) pb[outptr + incl - 1u] = (uint8_t)c;
            outptr += (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)last);
            p += last + 1u;
            if (ev) break;
        }
    } else if (staged) {
        for (uint32_t i = lane; i < ne / 4u; i += 64)
            ((uint32_t *)pb)[i] = __builtin_amdgcn_alignbyte(stg[i + 1u], stg[i], sh);
    } else {
        for (uint32_t i = lane; i < ne; i += 64) pb[i] = blob[d.dsd_prob_off + i];
    }
    __syncthreads();
    // running sums per bin, last bin first: lane l holds entries 4l .. 4l + 3 of the row
    for (uint32_t b = bins; b-- > 0;) {
        const uint32_t w = ((const uint32_t *)pb)[b * 64u + lane];
        uint4 v = make_uint4(w & 0xFFu, (w >> 8) & 0xFFu, (w >> 16) & 0xFFu, w >> 24);
        v.y += v.x;
        v.z += v.y;
        v.w += v.z;
        const uint32_t before = wave_incl_scan(v.w) - v.w;
        v.x = (v.x + before) & 0xFFFFu;
        v.y = (v.y + before) & 0xFFFFu;
        v.z = (v.z + before) & 0xFFFFu;
        v.w = (v.w + before) & 0xFFFFu;
        __builtin_amdgcn_wave_barrier();
        *(uint4 *)(tab + b * 256u + lane * 4u) = v;
    }
    __syncthreads();
}

// Mode 1: one wave per block, its tables staged in LDS first.  Launched over
// the mode-1 part of the DSD list (the list is sorted by kind);
// wv_decode_dsd_wave skips those blocks.  dsd_fast_v2 reads rows of u32
// cumulative counts (32 KiB at the framing's maximum of 32 bins).
constexpr uint32_t kDsdFastLds = 32u * 256u * 4u;
extern "C" __global__ void __launch_bounds__(64) wv_decode_dsd_fast(const BlockDesc *__restrict__ descs,
                                                                    const uint32_t *__restrict__ list,
                                                                    const uint8_t *__restrict__ blob,
                                                                    const uint8_t *__restrict__ tables,
                                                                    int32_t *__restrict__ out,
                                                                    uint32_t *__restrict__ status,
                                                                    uint32_t *__restrict__ mute_chunk,
                                                                    uint32_t mode) {
    __shared__ uint32_t tab[kDsdFastLds / 4];
    static_assert(kDsdStageAt * 4u + kDsdProbStage <= kDsdFastLds, "the stage lives in the row region");
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    // mode bit 2: only the blocks the row kernel (wv_dsd1_lane.hip) handed back (ST_REDO)
    if ((mode & 4u) && !(status[bi] & lane::ST_REDO)) return;
    if (d.inherit & INH_MEMBER) return;  // decoded by its chain's first block
    if (d.chain_len >= 2) {  // (the generic decode with the host's tables; tab: the ptable scratch)
        decode_dsd_chain(descs, bi, blob, tables, (int32_t *)tab, out, status, mute_chunk, mode);
        return;
    }
    const bool lead = threadIdx.x == 0;
    const uint32_t bins = (uint32_t)d.dsd_history_bins;
    DevStoreWave st{out + d.out_off, (uint64_t)d.pre_end * d.out_nch, lead};
    DsdResult r;
#if WV_M1_HOSTTAB  // measurement build only: the host framing's tables (host-framed blocks)
    {
        const uint16_t *sum16 = (const uint16_t *)(tables + d.dsd_table_off + (size_t)bins * 256u);
        const uint32_t ne = bins <= 32u ? bins * 256u : 0u;
        for (uint32_t i = threadIdx.x; i < ne; i += 64) tab[i] = sum16[i];
        __syncthreads();
    }
#else
    if (bins <= 32u) dsd_fast_tables(d, blob, bins, tab);
#endif
    // lane b: bin b's total and the reciprocal constants of dividing by it
    uint32_t vmag = 0, vsh1 = 0, vsh2 = 0;  // all zero for an empty bin (see dsd_fast_v2)
    if (threadIdx.x < bins && bins <= 32u) {
        const uint32_t dv = tab[threadIdx.x * 256u + 255u];
        if (dv) {
            const uint32_t l = dv > 1u ? 32u - (uint32_t)__clz(dv - 1u) : 0u;  // ceil(log2 dv)
            vmag = (uint32_t)(((((uint64_t)1 << l) - dv) << 32) / dv) + 1u;
            vsh1 = l ? 1u : 0u;
            vsh2 = l ? l - 1u : 0u;
        }
    }
    __syncthreads();
    if (bins > 32u)  // not produced by the framing (init_dsd_block_fast rejects > 5 history bits)
        r = decode_dsd_block(d, blob, tables, nullptr, st, g_dsd_ptables);
    else
        r = (d.flags & wvf::MONO_DATA) ? dsd_fast_v2<1>(d, blob, tab, vmag, vsh1, vsh2, st)
                                       : dsd_fast_v2<2>(d, blob, tab, vmag, vsh1, vsh2, st);
    if (lead) {
        status[bi] = d.fstatus | r.status | ((mode & 4u) ? (uint32_t)ST_REDONE : 0u);
        mute_chunk[bi] = r.mute_chunk;
    }
}

// one thread per DSD block; fills only for blocks that muted.  A false-stereo
// block whose final call failed its CRC (the mute set after that call's decode,
// DsdUtils.cs:99-119) returns before the stereo expansion: the call's values stay
// one per frame from its buffer position (dsd_fs_unexpand), and the second half of
// the expanded range keeps the caller's stale buffer where the fill does not reach
// it -- a block that starts inside its call (ST_NONDET)
__device__ __forceinline__ void dsd_fs_unexpand(const BlockDesc &d, uint32_t f, uint32_t len, int32_t *out,
                                                uint32_t &st) {
    const int64_t p = (int64_t)d.out_off + (int64_t)f * d.out_nch;
    for (int64_t k = 0; k < (int64_t)len; k++) out[p + k] = out[p + 2 * k];  // (ascending: reads ahead of writes)
    if (f == 0 && d.first_bsp > 0) st |= ST_NONDET;
}
extern "C" __global__ void __launch_bounds__(64) wv_dsd_fill(const BlockDesc *__restrict__ descs,
                                                             const uint32_t *__restrict__ list, uint32_t n,
                                                             uint32_t *__restrict__ status,
                                                             const uint32_t *__restrict__ mute_chunk,
                                                             int32_t *__restrict__ out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t bi = list[i];
    const BlockDesc &d = descs[bi];
    uint32_t st = status[bi];
    if (!(st & ST_DSD_MUTE)) return;
    const bool fs = (d.flags & wvf::FALSE_STEREO) && !(d.flags & wvf::MONO_FLAG) && d.nframes == d.block_samples;
    uint32_t f = 0, cl = d.first_chunk, mc = mute_chunk[bi];
    for (uint32_t ci = 0; f < d.nframes; ci++) {
        uint32_t len = cl < d.nframes - f ? cl : d.nframes - f;
        if (ci >= mc && f >= d.pre_end) {  // a seek's discard calls fill a buffer that is dropped
            if (fs && ci == mc && f + len == d.nframes) dsd_fs_unexpand(d, f, len, out, st);
            int64_t start = (int64_t)d.out_off + (int64_t)f * d.out_nch - (ci == 0 ? (int64_t)d.first_bsp : 0);
            for (int64_t k = 0; k < (int64_t)len * d.call_nch; k++) out[start + k] = 0x55;
        }
        f += len;
        cl = next_call_len(d, f);
    }
    status[bi] = st;
}

// read_decorr_weights / read_decorr_samples / read_entropy_vars /
// read_hybrid_profile (UnpackUtils.cs:196-360, WordsUtils.cs:75-187) for the
// reads the host framing deferred: job i applies its items, in stream order,
// to descriptor jobs[i].desc.  A few dozen bytes per block: latency, not
// bandwidth, so one lane per block and nothing staged.
extern "C" __global__ void __launch_bounds__(64) wv_meta_parse(BlockDesc *__restrict__ descs,
                                                               const MetaJob *__restrict__ jobs, uint32_t n,
                                                               const MetaItem *__restrict__ items,
                                                               const uint8_t *__restrict__ blob) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const MetaJob j = jobs[i];
    BlockDesc &d = descs[j.desc];
    for (uint32_t k = 0; k < j.count; k++) meta_apply(d, items[j.first + k], blob);
}

// WavpackFormatSamples (WavPackUtils.cs:288-341): one workgroup per segment of
// a file's int32 output; bytes_per_sample 1 (+128, or the raw byte with
// dsd), 2, 3 or 4, little-endian.  Memory-bound epilogue: 4 B read + bps B
// written per value.
extern "C" __global__ void __launch_bounds__(256) wv_format_pcm(const FormatSeg *__restrict__ segs,
                                                                const int32_t *__restrict__ in,
                                                                uint8_t *__restrict__ out, int dsd) {
    const FormatSeg s = segs[blockIdx.x];
    const int32_t *src = in + s.in_off;
    uint8_t *dst = out + s.out_off;
    for (uint32_t i = threadIdx.x; i < s.n; i += 256) {
        const int32_t t = src[i];
        switch (s.bps) {
        case 1: dst[i] = dsd ? (uint8_t)t : (uint8_t)(0xFF & (t + 128)); break;
        case 2: reinterpret_cast<uint16_t *>(dst)[i] = (uint16_t)t; break;
        case 3:
            dst[3 * (uint64_t)i] = (uint8_t)t;
            dst[3 * (uint64_t)i + 1] = (uint8_t)(t >> 8);
            dst[3 * (uint64_t)i + 2] = (uint8_t)(t >> 16);
            break;
        case 4: reinterpret_cast<int32_t *>(dst)[i] = t; break;
        default: break;  // the reference writes nothing for other widths
        }
    }
}

}  // namespace wvg

// ---------------------------------------------------------------------------
// two-wave PCM kernels, one instantiation per decorrelation term list
// (decoder order, i.e. the reverse of the encoder's; see wv_wave2.h)
// ---------------------------------------------------------------------------
namespace wvg {

template <int... Ts>
__global__ void __launch_bounds__(128) wv_pcm_2wave(const BlockDesc *__restrict__ descs,
                                                    const uint32_t *__restrict__ list,
                                                    const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                    uint32_t *__restrict__ status, uint32_t *__restrict__ aux) {
    w2::block_2wave<Ts...>(descs, list, blob, out, status, aux);
}

// the two-wave kernel over the blocks the lane-per-block kernel (wv_lane.hip)
// handed back (ST_REDO; every other block's workgroup exits at once)
template <int... Ts>
__global__ void __launch_bounds__(128) wv_pcm_2wave_redo(const BlockDesc *__restrict__ descs,
                                                         const uint32_t *__restrict__ list,
                                                         const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                         uint32_t *__restrict__ status, uint32_t *__restrict__ aux) {
    if (!(status[list[blockIdx.x]] & lane::ST_REDO)) return;
    w2::block_2wave<Ts...>(descs, list, blob, out, status, aux);
    if (threadIdx.x == 64) status[list[blockIdx.x]] |= ST_REDONE;  // (the lane that stored the status: wave 1's lane 0)
}

// pipelined reconstruction (wv_pipe.h): any term list, one kernel per "has -1/-2"
template <bool NEG12>
__global__ void __launch_bounds__(128) wv_pcm_pipe(const BlockDesc *__restrict__ descs,
                                                   const uint32_t *__restrict__ list,
                                                   const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                   uint32_t *__restrict__ status, uint32_t *__restrict__ aux) {
    w2::block_pipe<NEG12>(descs, list, blob, out, status, aux);
}
// ... over the blocks a lane kernel handed back, for the lane-only term lists
template <bool NEG12>
__global__ void __launch_bounds__(128) wv_pcm_pipe_redo(const BlockDesc *__restrict__ descs,
                                                        const uint32_t *__restrict__ list,
                                                        const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                        uint32_t *__restrict__ status, uint32_t *__restrict__ aux) {
    if (!(status[list[blockIdx.x]] & lane::ST_REDO)) return;
    w2::block_pipe<NEG12>(descs, list, blob, out, status, aux);
    if (threadIdx.x == 64) status[list[blockIdx.x]] |= ST_REDONE;  // (the lane that stored the status: wave 1's lane 0)
}

// the shallow lists WavPack writes most (decoder order, the reverse of the
// encoder's): each is a compile-time VALU chain (wv_wave2.h); deeper or other
// lists run the pipelined kernel (WVG_TS_*: wv_lane.h)

static const int8_t kTermSets[][17] = {
    // {count, terms...}
    {2, WVG_TS_FAST},
    {5, WVG_TS_DEFAULT},
    {5, WVG_TS_M5},
};
constexpr int kNumTermSets = 3;

// launch groups 0..kNumTermSets-1: the two-wave kernels with a compile-time term
// list; kPipe / kPipe + 1: the pipelined kernel without / with stereo -1/-2 terms
constexpr int kPipe = 3;
static_assert(kNumTermSets <= kPipe, "term-set slots");

// lists with a lane-kernel specialisation only (launch group kLaneBase + i): the
// lane kernel when the batch asks for it, else the pipelined kernel.  WavPack's
// 16-term 'high' lists: stereo (C3's, C5's 24-bit stereo) and mono (C5's 24-bit
// mono).  The mono lane kernel also takes the M5 set's blocks (WavPack's mono
// default list: C5's 16-bit mono and false-stereo files).
static const int8_t kLaneSets[][17] = {
    {16, WVG_TS_HIGH16},
    {16, WVG_TS_MONO_HIGH16},
};
constexpr int kNumLaneSets = 2;
constexpr int kLaneBase = kPipe + 2;
// hybrid stereo blocks of the default list (HYBRID_BITRATE, no HYBRID_BALANCE, not
// int32: C4's float hybrid): the hybrid lane kernel when the batch asks for it,
// else the default list's two-wave kernel
constexpr int kHyDefault = kLaneBase + kNumLaneSets;
static_assert(kHyDefault < 8, "launch groups (wv_api.cpp kMaxTermSets)");
static const bool kLaneSetMono[kNumLaneSets] = {false, true};
static const bool kLaneSetNeg12[kNumLaneSets] = {true, false};

// which two-wave kernel decodes this block (-1: the generic wave kernel, for
// int32 + wvx, .wvc, exact-float and chained blocks).  prefer_pipe 2: every list goes to the pipelined kernel
// (A/B tests)
// the launch groups whose lane kernel reads the list at run time (wv_pcm_lane_rt / _rt3): the
// pipelined kernel's lists and the 16-term lists (the host orders their lane lists by list)
bool lane_rt_group(int ts) { return ts == kPipe || ts == kPipe + 1 || (ts >= kLaneBase && ts < kLaneBase + kNumLaneSets); }

int term_set_of(const BlockDesc &d, int prefer_pipe) {
    using namespace wvf;
    if (d.kind != KIND_PCM) return -1;
    if (d.chain_len >= 2 || (d.inherit & INH_MEMBER)) return -1;  // sticky-state chain (wv_decode_pcm_wave)
    if (d.wvx_state & 0x100) return -1;  // int32 + wvx fixup reads a second stream
    if (d.wvc_len) return -1;            // .wvc correction: a second stream read per hybrid word
    if (d.xfloat) return -1;             // exact float: WavPack 4's float_values over the wvx stream
    // FALSE_STEREO with MONO_FLAG, or a block whose ints a frame differ from the file's:
    // the layout rules of decode_pcm_run (malformed files only)
    if ((d.flags & FALSE_STEREO) && (d.flags & MONO_FLAG)) return -1;
    if ((((d.flags & MONO_FLAG) && !(d.flags & FALSE_STEREO)) ? 1u : 2u) != d.out_nch) return -1;
    const bool mono = (d.flags & MONO_DATA) != 0;
    if (d.num_terms < 0 || d.num_terms > MAXP) return -1;
    bool neg12 = false;
    for (int i = 0; i < d.num_terms; i++) {
        neg12 |= !mono && (d.term[i] == -1 || d.term[i] == -2);
        if (!mono && d.term[i] == 0) return -1;  // term 0's call-position rule: pass_stereo's `cont`
    }
    const int pipe = kPipe + (neg12 ? 1 : 0);
    if (prefer_pipe >= 2) return pipe;
    for (int s = 0; s < kNumTermSets; s++) {
        if (kTermSets[s][0] != d.num_terms) continue;
        bool ok = true;
        for (int i = 0; i < d.num_terms && ok; i++) {
            int t = kTermSets[s][1 + i];
            if (t != d.term[i]) ok = false;
            if (mono && t < 0) ok = false;
        }
        if (ok) {
            if (d.flags & HYBRID_FLAG) {
                // hybrid: stereo default-list blocks on their own lane kernel (kHyDefault; with or
                // without HYBRID_BITRATE, integer, float or int32 without wvx), every other one
                // with the run-time list lanes (or the pipelined kernel)
                if (s == 1 && !mono) return kHyDefault;
                return pipe;
            }
            return s;
        }
    }
    {
        for (int s = 0; s < kNumLaneSets; s++) {
            if (kLaneSetMono[s] != mono || kLaneSets[s][0] != d.num_terms) continue;
            bool ok = true;
            for (int i = 0; i < d.num_terms && ok; i++) ok = kLaneSets[s][1 + i] == d.term[i];
            if (ok) return kLaneBase + s;
        }
    }
    return pipe;
}

hipError_t launch_2wave(int ts, const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                        int32_t *out, uint32_t *status, uint32_t *aux, hipStream_t s, int lane_mode,
                        const uint32_t *lane_list, uint32_t lane_n, uint32_t *lane_dbg) {
    if (!n) return hipSuccess;
    dim3 g(n), b(128);
    if (ts >= kLaneBase && ts < kLaneBase + kNumLaneSets) {
        const bool neg12 = kLaneSetNeg12[ts - kLaneBase];
        if (!lane_mode) {
            if (neg12) hipLaunchKernelGGL((wv_pcm_pipe<true>), g, b, 0, s, descs, list, blob, out, status, aux);
            else hipLaunchKernelGGL((wv_pcm_pipe<false>), g, b, 0, s, descs, list, blob, out, status, aux);
            return hipGetLastError();
        }
        dim3 gl((lane_n + 64 * lane::LPAIRS - 1) / (64 * lane::LPAIRS)), bl(64 * lane::LPAIRS * 2);
        // the 16-term lists on the run-time list kernel (wv_pcm_lane_rt3): its reconstruction
        // pipeline of three waves beats the one-wave compile-time chain -- C3 (1,024 blocks, 20
        // in flight) 32,700 vs 28,900 Mframes/s, 22.1 vs 24.8 ms alone (profiles/r05_lists_rates.jsonl);
        // WVG_LANE_HIGH16=ct: the compile-time instantiations (A/B)
        static const bool high_rt = !(getenv("WVG_LANE_HIGH16") && strcmp(getenv("WVG_LANE_HIGH16"), "ct") == 0);
        const int which = high_rt ? LANE_RT : (ts - kLaneBase == 0 ? LANE_HIGH16 : LANE_MONO_HIGH16);
        if (hipError_t e = launch_lane(which, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
        if (lane_mode != 2) {
            if (neg12) hipLaunchKernelGGL((wv_pcm_pipe_redo<true>), g, b, 0, s, descs, list, blob, out, status, aux);
            else hipLaunchKernelGGL((wv_pcm_pipe_redo<false>), g, b, 0, s, descs, list, blob, out, status, aux);
        }
        return hipGetLastError();
    }
    if (ts == kHyDefault) {
        if (lane_mode) {
            dim3 gl((lane_n + 64 * lane::LPAIRS - 1) / (64 * lane::LPAIRS)), bl(64 * lane::LPAIRS * 2);
            if (hipError_t e = launch_lane(LANE_HY_DEFAULT, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
            if (lane_mode != 2) hipLaunchKernelGGL((wv_pcm_2wave_redo<WVG_TS_DEFAULT>), g, b, 0, s, descs, list, blob, out, status, aux);
        } else {
            hipLaunchKernelGGL((wv_pcm_2wave<WVG_TS_DEFAULT>), g, b, 0, s, descs, list, blob, out, status, aux);
        }
        return hipGetLastError();
    }
    if (lane_mode && ts < kNumTermSets) {
        dim3 gl((lane_n + 64 * lane::LPAIRS - 1) / (64 * lane::LPAIRS)), bl(64 * lane::LPAIRS * 2);
        switch (ts) {
        case 0:
            if (hipError_t e = launch_lane(LANE_FAST, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
            if (lane_mode != 2)  // 2: the lane kernel alone (diagnostics: ST_REDO stays in the status)
                hipLaunchKernelGGL((wv_pcm_2wave_redo<WVG_TS_FAST>), g, b, 0, s, descs, list, blob, out, status, aux);
            break;
        case 1:
            if (hipError_t e = launch_lane(LANE_DEFAULT, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
            if (lane_mode != 2)  // 2: the lane kernel alone (diagnostics: ST_REDO stays in the status)
                hipLaunchKernelGGL((wv_pcm_2wave_redo<WVG_TS_DEFAULT>), g, b, 0, s, descs, list, blob, out, status, aux);
            break;
        case 2:
            // (the mono default list: its blocks are mono or false stereo; a stereo block goes to the redo)
            if (hipError_t e = launch_lane(LANE_M5, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
            if (lane_mode != 2)  // 2: the lane kernel alone (diagnostics: ST_REDO stays in the status)
                hipLaunchKernelGGL((wv_pcm_2wave_redo<WVG_TS_M5>), g, b, 0, s, descs, list, blob, out, status, aux);
            break;
        }
        return hipGetLastError();
    }
    if (lane_mode && (ts == kPipe || ts == kPipe + 1)) {
        // every other lossless list of up to 16 terms: the run-time list lane kernel (the
        // host orders its lane list by list, wv_api.cpp build_lane_orders), then the
        // pipelined kernel over its hand-backs
        dim3 gl((lane_n + 64 * lane::LPAIRS - 1) / (64 * lane::LPAIRS)), bl(64 * lane::LPAIRS * 2);
        if (hipError_t e = launch_lane(LANE_RT, gl, bl, s, descs, lane_list, lane_n, blob, out, status, lane_dbg); e != hipSuccess) return e;
        if (lane_mode != 2) {
            if (ts == kPipe + 1) hipLaunchKernelGGL((wv_pcm_pipe_redo<true>), g, b, 0, s, descs, list, blob, out, status, aux);
            else hipLaunchKernelGGL((wv_pcm_pipe_redo<false>), g, b, 0, s, descs, list, blob, out, status, aux);
        }
        return hipGetLastError();
    }
    switch (ts) {
    case 0: hipLaunchKernelGGL((wv_pcm_2wave<WVG_TS_FAST>), g, b, 0, s, descs, list, blob, out, status, aux); break;
    case 1: hipLaunchKernelGGL((wv_pcm_2wave<WVG_TS_DEFAULT>), g, b, 0, s, descs, list, blob, out, status, aux); break;
    case 2: hipLaunchKernelGGL((wv_pcm_2wave<WVG_TS_M5>), g, b, 0, s, descs, list, blob, out, status, aux); break;
    case kPipe: hipLaunchKernelGGL((wv_pcm_pipe<false>), g, b, 0, s, descs, list, blob, out, status, aux); break;
    case kPipe + 1: hipLaunchKernelGGL((wv_pcm_pipe<true>), g, b, 0, s, descs, list, blob, out, status, aux); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace wvg

// ---------------------------------------------------------------------------
// host launchers (called from wv_api.cpp)
// ---------------------------------------------------------------------------
namespace wvg {

// PCM blocks without a two-wave instantiation (generic wave kernel) on s_pcm;
// DSD blocks: the mode-1 range [fast_lo, fast_lo + n_fast) of the kind-sorted
// list by wv_decode_dsd_fast on s_fast, every other DSD block by one
// wv_decode_dsd_wave launch on s_dsd (mute fills: launch_dsd_fill, after the join)
// With lane_mode, the mode-3 range [high_lo, n_dsd) (stereo first, then n_high_mono
// mono blocks) goes to the lane-per-block kernel (wv_dsd_lane.hip) after the wave
// kernel's other blocks, and the wave kernel then decodes what it handed back; with
// lane_mode_fast, the mode-1 range (stereo first, then n_fast_mono mono blocks) to the
// 16-lane row kernel (wv_dsd1_lane.hip), its hand-backs to wv_decode_dsd_fast.
hipError_t launch_decode(const BlockDesc *descs, const uint32_t *pcm_list, uint32_t n_pcm, const uint32_t *dsd_list,
                         uint32_t n_dsd, uint32_t fast_lo, uint32_t n_fast, const uint8_t *blob, const uint8_t *tables,
                         int32_t *out, uint32_t *status, uint32_t *aux, hipStream_t s_pcm, hipStream_t s_dsd,
                         hipStream_t s_fast, int lane_mode, uint32_t high_lo, uint32_t n_high_mono,
                         int lane_mode_fast, uint32_t n_fast_mono, int lane_mode_wvc, uint32_t n_pcm_wvc) {
    // the DSD kernels first: their blocks are the batch's longest serial chains
    const uint32_t skip = n_fast ? 1u : 0u;
    const uint32_t n_high = lane_mode ? n_dsd - high_lo : 0u;
    if (n_dsd > n_fast + n_high) {
        hipLaunchKernelGGL(wv_decode_dsd_wave, dim3(n_dsd - n_high), dim3(64), 0, s_dsd, descs, dsd_list, blob, tables,
                           out, status, aux, skip | (n_high ? 2u : 0u));
    }
    if (n_high) {
        if (hipError_t e = launch_dsd3_lane(descs, dsd_list + high_lo, n_high, blob, dsd_ptables_device(), out, status,
                                            aux, n_high_mono, s_dsd);
            e != hipSuccess)
            return e;
        if (lane_mode != 2)  // 2: the lane kernel alone (diagnostics: ST_REDO stays in the status)
            hipLaunchKernelGGL(wv_decode_dsd_wave, dim3(n_high), dim3(64), 0, s_dsd, descs, dsd_list + high_lo, blob,
                               tables, out, status, aux, 4u);
    }
    if (n_fast) {
        const uint32_t *fl = dsd_list + fast_lo;
        if (lane_mode_fast) {
            // mode 1 on rows of 16 lanes (wv_dsd1_lane.hip), then its hand-backs one wave per block
            if (hipError_t e = launch_dsd1_lane(descs, fl, n_fast, blob, out, status, aux, n_fast_mono, s_fast);
                e != hipSuccess)
                return e;
            if (lane_mode_fast != 2)  // 2: the row kernel alone (diagnostics: ST_REDO stays in the status)
                hipLaunchKernelGGL(wv_decode_dsd_fast, dim3(n_fast), dim3(64), 0, s_fast, descs, fl, blob, tables, out,
                                   status, aux, 4u);
        } else {
            hipLaunchKernelGGL(wv_decode_dsd_fast, dim3(n_fast), dim3(64), 0, s_fast, descs, fl, blob, tables, out,
                               status, aux, 0u);
        }
    }
    if (n_pcm && lane_mode_wvc && n_pcm_wvc) {
        // the list's tail: hybrid default-list blocks with a .wvc stream on the .wvc lane
        // kernel, then what it handed back on the generic kernel (the head as usual)
        const uint32_t nh = n_pcm - n_pcm_wvc;
        const uint32_t *tl = pcm_list + nh;
        dim3 gl((n_pcm_wvc + 64 * lane::LPAIRS - 1) / (64 * lane::LPAIRS)), bl(64 * lane::LPAIRS * 2);
        if (hipError_t e = launch_lane(LANE_HY_WVC, gl, bl, s_pcm, descs, tl, n_pcm_wvc, blob, out, status, nullptr);
            e != hipSuccess)
            return e;
        if (nh)
            hipLaunchKernelGGL(wv_decode_pcm_wave, dim3(nh), dim3(64), 0, s_pcm, descs, pcm_list, blob, out, status, aux,
                               0u);
        if (lane_mode_wvc != 2)  // 2: the lane kernel alone (diagnostics: ST_REDO stays in the status)
            hipLaunchKernelGGL(wv_decode_pcm_wave, dim3(n_pcm_wvc), dim3(64), 0, s_pcm, descs, tl, blob, out, status,
                               aux, 4u);
    } else if (n_pcm) {
        hipLaunchKernelGGL(wv_decode_pcm_wave, dim3(n_pcm), dim3(64), 0, s_pcm, descs, pcm_list, blob, out, status, aux,
                           0u);
    }
    return hipGetLastError();
}

// the 0x55 mute fills of every DSD block (quirk B-9), on the batch stream after
// every decode launch has joined it: a fill starts at its call's buffer start,
// i.e. inside the output of earlier blocks of the same call, which may be PCM
// or DSD blocks decoded on other streams
hipError_t launch_dsd_fill(const BlockDesc *descs, const uint32_t *dsd_list, uint32_t n_dsd, uint32_t *status,
                           const uint32_t *aux, int32_t *out, hipStream_t s) {
    if (!n_dsd) return hipSuccess;
    hipLaunchKernelGGL(wv_dsd_fill, dim3((n_dsd + 63) / 64), dim3(64), 0, s, descs, dsd_list, n_dsd, status, aux, out);
    return hipGetLastError();
}

hipError_t launch_meta(BlockDesc *descs, const MetaJob *jobs, uint32_t njobs, const MetaItem *items, const uint8_t *blob,
                       hipStream_t s) {
    if (!njobs) return hipSuccess;
    hipLaunchKernelGGL(wv_meta_parse, dim3((njobs + 63) / 64), dim3(64), 0, s, descs, jobs, njobs, items, blob);
    return hipGetLastError();
}

// the gap zero-fills of a decode (ZeroSeg, wv_framing.h): one workgroup per segment
__global__ void __launch_bounds__(256) wv_zero_fill(const ZeroSeg *__restrict__ segs, int32_t *__restrict__ out) {
    const ZeroSeg z = segs[blockIdx.x];
    for (uint64_t i = threadIdx.x; i < z.n; i += 256) out[z.off + i] = 0;
}

hipError_t launch_zero_fill(const ZeroSeg *segs, uint32_t nseg, int32_t *out, hipStream_t s) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(wv_zero_fill, dim3(nseg), dim3(256), 0, s, segs, out);
    return hipGetLastError();
}

hipError_t launch_format(const FormatSeg *segs, uint32_t nseg, const int32_t *in, uint8_t *out, int dsd, hipStream_t s) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(wv_format_pcm, dim3(nseg), dim3(256), 0, s, segs, in, out, dsd);
    return hipGetLastError();
}

// n bytes from HBM into page-locked host memory by the CUs (16 B per lane, the
// stores crossing PCIe as full lines): the async PCM download, a kernel in the
// batch stream's order rather than a DMA-engine copy, whose dependency on the
// format kernel the runtime resolves on the host (pipe2_probe: a thread issuing
// request k+1 blocked for milliseconds behind request k's queued copy)
extern "C" __global__ void __launch_bounds__(256) wv_copy_to_host(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                                  uint64_t n16, const uint8_t *__restrict__ tsrc,
                                                                  uint8_t *__restrict__ tdst, uint32_t ntail) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < ntail) tdst[threadIdx.x] = tsrc[threadIdx.x];
}

hipError_t launch_copy_to_host(const uint8_t *src, uint8_t *dst, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t n16 = n / 16;
    const uint32_t ntail = (uint32_t)(n - n16 * 16);
    // 1,024 workgroups (4 per CU): enough stores in flight to cover the PCIe round trip
    hipLaunchKernelGGL(wv_copy_to_host, dim3(1024), dim3(256), 0, s, (const uint4 *)src, (uint4 *)dst, n16,
                       src + n16 * 16, dst + n16 * 16, ntail);
    return hipGetLastError();
}

}  // namespace wvg
