// wv_dsd_lane.hip -- DSD mode 3 (DsdUtils.init_dsd_block_high + decode_high,
// DsdUtils.cs:321-493) with one lane per block: the throughput kernel for
// batches with many mode-3 blocks (wvg_batch_set_kernel(WVG_KERNEL_LANE)).
//
// A mode-3 block is one serial range-coder chain (8 binary decisions per
// channel byte, each reading and updating an adaptive 256-entry probability
// table), so the wave-per-block kernel (wv_decode.hip, dsd_high_v2) spends a
// whole wave on one chain.  Here each lane of a wave owns one block: its range
// coder (low, high, value), both channels' filter states and its probability
// table, which sits in LDS interleaved by lane (entry e of lane l at
// (e * 64 + l) * 4: every lane's read hits bank l, and the address of the entry a
// filter value selects is one v_and_or).  One VALU instruction moves 64 chains.
//
// Payload bytes come from a per-lane 64-bit big-endian window refilled a dword at
// a time from a dword loaded one refill ahead (global loads, one per 4 bytes),
// every 4 decisions (>= 5 bytes then): a block's first frames, while its filters
// adapt, take up to ~4 bytes per 4 decisions.  A lane whose window runs dry
// (checked after every decision), or a block outside the kernel's scope (a seek's
// discard calls, state from an earlier block, a framing verdict), is marked
// ST_REDO and decoded again right after by the wave-per-block kernel, so results
// are exactly the wave kernel's, which the GPU tests hold against the oracle.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "wv_desc.h"
#include "wv_format.h"

namespace wvg {
namespace dlane {

constexpr uint32_t ST_REDO = 1u << 15;  // as wv_lane.h: decode this block again (wave kernel)
constexpr int32_t kUp = 0x010000FE, kDown = 0x00010000;  // DsdUtils.cs UP / DOWN

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// per-lane payload window: byte bp of the payload in bits 63..56 of win, `avail`
// bytes valid, nxt / nxt2 = the two dwords after them (loaded two refills ahead: a
// refill comes every ~600 cycles, a global load can take longer)
struct Win {
    const uint32_t *w;
    uint64_t win;
    int32_t avail;
    uint32_t ni, nxt, nxt2;
    __device__ __forceinline__ void init(const uint8_t *p) {
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
        w = (const uint32_t *)(p - sh);
        win = (uint64_t)bswap(w[0]) << (32u + 8u * sh);
        avail = 4 - (int32_t)sh;
        nxt = w[1];
        nxt2 = w[2];
        ni = 3;
        refill();
    }
    // avail <= 4: four more bytes below the valid ones (branch-free: a lane with
    // more keeps its window and its read-ahead dwords)
    __device__ __forceinline__ void refill() {
        const bool m = avail <= 4;
        const uint32_t sh = (uint32_t)(32 - 8 * (m ? avail : 0)) & 63u;
        win |= m ? (uint64_t)bswap(nxt) << sh : 0ull;
        avail += m ? 4 : 0;
        const uint32_t nn = w[ni];  // (read every time: the address is always inside the blob's tail)
        nxt = m ? nxt2 : nxt;
        nxt2 = m ? nn : nxt2;
        ni += m ? 1u : 0u;
    }
};

// one range-coder decision of decode_high (DsdUtils.cs:409-429) and the
// renormalisation after it (the byte loop as one shift of n = leading zero bytes of
// high ^ low, capped by the bytes left): returns filter0 (-1 when value <= split)
__device__ __forceinline__ int32_t decide(uint32_t &low, uint32_t &high, uint32_t &value, uint32_t pv, Win &src,
                                          uint32_t &left) {
    const uint32_t split = low + __umul24((high - low) >> 8, pv >> 16);  // (24-bit by 9-bit: exact)
    const bool zero = value <= split;
    high = zero ? split : high;
    low = zero ? low : split + 1u;
    // bytes to shift out: leading zero bytes of high ^ low (v_ffbh_u32 of 0 is ~0: 4 after
    // the cap), at most the bytes left
    uint32_t lz;
    asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(high ^ low));
    const uint32_t n = min(min(lz >> 3, 4u), left);
    const uint32_t s = n << 3;  // 0..32
    value = (uint32_t)(((((uint64_t)value << 32) | (src.win >> 32)) << s) >> 32);
    high = (uint32_t)(((((uint64_t)high << 32) | 0xFFFFFFFFull) << s) >> 32);
    low = (uint32_t)(((uint64_t)low << s) & 0xFFFFFFFFull);
    src.win <<= s;
    src.avail -= (int32_t)n;
    left -= n;
    return zero ? -1 : 0;
}

// a channel's filter state (DSDfilters: value q0, filter1..6 q2..q7, factor q8)
struct Filt {
    int32_t q0, q2, q3, q4, q5, q6, q7, q8, byte;
};
__device__ __forceinline__ int32_t fval(const Filt &f) {  // filter1 - filter5 + (filter6 * factor >> 2)
    return (f.q2 - f.q6) + (__mul24(f.q7, f.q8) >> 2);
}
// the filter update after a decision (DsdUtils.cs:430-441); filter6 and factor stay
// far inside 24 bits for any stream (convex updates of 0 / 2^20; the factor decays
// 1/1024 per byte), so the products are 24-bit multiplies with C#'s low 32 bits
__device__ __forceinline__ void fupd(Filt &f, int32_t f0) {
    const int32_t v = f.q0 + (f.q7 << 3);
    const int32_t t = f.q0 - (f.q7 << 3);          // value - filter6 * 16, after the += filter6 * 8
    f.byte = (f.byte << 1) | (f0 & 1);
    f.q8 += (((v ^ f0) >> 31) | 1) & ((v ^ t) >> 31);
    const int32_t x = f0 & (1 << 20);
    f.q2 += (x - f.q2) >> 6;
    f.q3 += (x - f.q3) >> 4;
    f.q4 += (f.q3 - f.q4) >> 4;
    f.q5 += (f.q4 - f.q5) >> 4;
    const int32_t dd = (f.q5 - f.q6) >> 4;
    f.q6 += dd;
    f.q7 += (dd - f.q7) >> 3;
    f.q0 = fval(f);
}

// can this lane decode block d exactly (else ST_REDO)?  CH: channels decoded
template <int CH>
__device__ __forceinline__ bool dsd3_ok(const BlockDesc &d) {
    using namespace wvf;
    if (d.kind != KIND_DSD_HIGH) return false;
    if (((d.flags & MONO_DATA) ? 1 : 2) != CH) return false;
    if (CH == 2 && (d.flags & FALSE_STEREO)) return false;
    // the lane stores och ints a frame: they must be the file's (a FALSE_STEREO block in a
    // 1-int file would write past its range)
    if (((CH == 2 || (d.flags & FALSE_STEREO)) ? 2u : 1u) != d.out_nch) return false;
    if (d.inherit || d.chain_len >= 2 || d.pre_end || d.fstatus) return false;
    if (d.dsd_data_len < 4u) return false;
    return true;
}

// One workgroup = one wave = 64 blocks; the probability tables take 64 KiB of
// LDS, so two waves share a CU (on two of its SIMDs).
template <int CH>
__device__ __forceinline__ void dsd3_lanes(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                           uint32_t n, const uint8_t *__restrict__ blob,
                                           const int32_t *__restrict__ ptables, int32_t *__restrict__ out,
                                           uint32_t *__restrict__ status, uint32_t *__restrict__ mute_chunk) {
    using namespace wvf;
    __shared__ int32_t pt[256 * 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t li = blockIdx.x * 64u + lane;
    const bool inl = li < n;
    const uint32_t bi = inl ? list[li] : 0u;
    const BlockDesc &d = descs[bi];
    const bool ok = inl && dsd3_ok<CH>(d);
    if (inl && !ok) status[bi] = ST_REDO | (1u << 16);
    const uint32_t nfr = ok ? d.nframes : 0u;
    // the wave runs to its longest block (uniform loop; finished lanes idle along)
    uint32_t nmax = nfr;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off));
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    if (nmax == 0u) return;
    // this lane's probability table: the block's starting row (init_ptable for its rate_i)
    uint8_t *ptb = (uint8_t *)pt;
    const uint32_t col = lane * 4u;
    {
        const int32_t *row = ptables + (uint32_t)(ok ? (d.dsd_rate_i & 255) : 0) * 256u;
        for (uint32_t e = 0; e < 256u; e++) *(int32_t *)(ptb + (e << 8) + col) = row[e];
    }
    Win src;
    src.init(blob + (ok ? d.bits_off : 0));
    uint32_t left = ok ? d.dsd_data_len : 4u;
    uint32_t low = 0u, high = 0xFFFFFFFFu, value = 0u;
    value = (uint32_t)(src.win >> 32);  // init_dsd_block_high's 4 value bytes
    src.win <<= 32;
    src.avail -= 4;
    left -= 4u;
    src.refill();
    Filt f[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) {
        f[c].q2 = d.dsd_filters[c][0];
        f[c].q3 = d.dsd_filters[c][1];
        f[c].q4 = d.dsd_filters[c][2];
        f[c].q5 = d.dsd_filters[c][3];
        f[c].q6 = d.dsd_filters[c][4];
        f[c].q7 = 0;
        f[c].q8 = d.dsd_filters[c][5];
        f[c].q0 = fval(f[c]);
        f[c].byte = 0;
    }
    const bool fst = (d.flags & FALSE_STEREO) != 0;
    const uint32_t och = (CH == 2 || fst) ? 2u : 1u;
    int32_t *o = out + d.out_off;
    int32_t crc = -1;
    int32_t dry = 0;  // least window bytes seen (< 0: the window ran dry, ST_REDO)
    __syncthreads();
    for (uint32_t t = 0; t < nmax; t++) {
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            // (a refill every 4 decisions: a block's first frames, before the filters
            // adapt, can take 4 bytes per 4 decisions)
            if (CH == 2 ? (bit & 1) == 0 && bit != 0 : bit == 4) src.refill();
            // both channels' entries first (each depends on its own filter only)
            uint32_t a[CH];
            int32_t pv[CH];
#pragma unroll
            for (int c = 0; c < CH; c++) {
                a[c] = ((uint32_t)f[c].q0 & 0xFF00u) | col;
                pv[c] = *(const int32_t *)(ptb + a[c]);
            }
            int32_t f0[CH], nv[CH];
#pragma unroll
            for (int c = 0; c < CH; c++) {
                // channel 1 takes the entry channel 0 just updated when both chose it
                // (forwarded; its store then lands after channel 0's)
                if (CH == 2 && c == 1) pv[CH - 1] = a[CH - 1] == a[0] ? nv[0] : pv[CH - 1];
                f0[c] = decide(low, high, value, (uint32_t)pv[c], src, left);
                dry = min(dry, t < nfr ? src.avail : 0);  // (a half frame past the window: its refill comes too late)
                nv[c] = pv[c] + (((f0[c] ? kUp : kDown) - pv[c]) >> 8);
                *(int32_t *)(ptb + a[c]) = nv[c];
            }
#pragma unroll
            for (int c = 0; c < CH; c++) fupd(f[c], f0[c]);
        }
        src.refill();
        // the frame's bytes, CRC (crc += 2 crc + v per value), factor decay (:484-492)
        int32_t v[CH];
#pragma unroll
        for (int c = 0; c < CH; c++) {
            v[c] = f[c].byte & 0xFF;
            crc = t < nfr ? crc * 3 + v[c] : crc;  // (a lane past its block's end idles along)
            f[c].q8 -= (f[c].q8 + 512) >> 10;
            f[c].q0 = fval(f[c]);  // (the next frame's value, :395-396, with the decayed factor)
        }
        if (t < nfr) {
            if (och == 2u) {  // (two dword stores: a file's output may start at an odd int)
                o[2u * t] = v[0];
                o[2u * t + 1u] = v[CH - 1];
            }
            else o[t] = v[0];
        }
    }
    if (!ok) return;
    uint32_t st = 0;
    if (dry < 0) {
        status[bi] = ST_REDO | (64u << 16);
        return;
    }
    if (d.nframes == d.block_samples) {
        st |= ST_CRC_CHECKED;
        if (crc != d.crc) {
            // DsdUtils.cs:99-117: the final call mutes -- 0x55 from the caller's buffer
            // start, and a false-stereo block's values left unexpanded -- the wave kernel's
            // call-by-call output; a corrupt block is rare: decoded again there
            status[bi] = ST_REDO | (8u << 16);
            return;
        }
    }
    status[bi] = st;
}

// ---------------------------------------------------------------------------
// Stereo blocks on lane pairs (round 6): lane 2j runs channel 0 of block j, lane
// 2j + 1 channel 1.  The range coder (low / high / value, the payload window) is
// one serial chain through both channels' decisions, so both lanes of a pair run
// it -- the same instructions, in parallel -- while each lane runs only its own
// channel's filter update, which in the one-lane kernel was half of a bit pair's
// instructions.  The pair's two table entries come from one LDS read (each lane
// reads its channel's entry, DPP quad_perm broadcasts give both lanes both), and
// each lane writes back its channel's updated entry (channel 0's when both chose
// the same entry is superseded by channel 1's, so both lanes write that one).
// ---------------------------------------------------------------------------

// quad_perm DPP moves within a lane pair: [1,0,3,2] swap, [0,0,2,2] even, [1,1,3,3] odd
__device__ __forceinline__ int32_t qp_swap(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int32_t qp_even(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xA0, 0xF, 0xF, false); }
__device__ __forceinline__ int32_t qp_odd(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xF5, 0xF, 0xF, false); }

// The payload window of a pair: as Win, with the valid byte count kept as
// base8 + left8 (bits; both fall by the same shift at every decision, so only the
// bits left in the block are counted per decision and the window's fill is
// recovered at each refill).
struct Win8 {
    const uint32_t *w;
    uint64_t win;
    int32_t base8;
    uint32_t ni, nxt, nxt2;
    __device__ __forceinline__ void init(const uint8_t *p, uint32_t left8) {
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
        w = (const uint32_t *)(p - sh);
        win = (uint64_t)bswap(w[0]) << (32u + 8u * sh);
        base8 = 8 * (4 - (int32_t)sh) - (int32_t)left8;
        nxt = w[1];
        nxt2 = w[2];
        ni = 3;
        refill(left8);
    }
    // returns the valid bits before the refill (< 0: the window ran dry since the last one)
    __device__ __forceinline__ int32_t refill(uint32_t left8) {
        const int32_t av = base8 + (int32_t)left8;
        const bool m = av <= 32;
        const uint32_t sh = (uint32_t)(32 - (m ? av : 0)) & 63u;
        win |= m ? (uint64_t)bswap(nxt) << sh : 0ull;
        base8 += m ? 32 : 0;
        const uint32_t nn = w[ni];  // (inside the blob's tail: ni stops advancing once left8 is 0)
        nxt = m ? nxt2 : nxt;
        nxt2 = m ? nn : nxt2;
        ni += m ? 1u : 0u;
        return av;
    }
};

// decide() with the shift in bits and only left8 counted (see Win8); p16 = the entry >> 16
__device__ __forceinline__ bool decide8p(uint64_t &lowp, uint32_t &high, uint32_t &value, uint64_t &win,
                                         uint32_t &left8, uint32_t p16) {
    // lowp: low in its low half, the high half undefined (the shift below leaves its
    // low 32 bits right whatever it holds, so no register pair is rebuilt per decision)
    uint32_t low = (uint32_t)lowp;
    const uint32_t split = low + __umul24((high - low) >> 8, p16);
    const bool zero = value <= split;
    high = zero ? split : high;
    low = zero ? low : split + 1u;
    uint32_t lz;
    asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(high ^ low));
    const uint32_t s = min(min(lz & ~7u, 32u), left8);  // (ffbh of 0 is ~0: 32 after the cap)
    value = (uint32_t)(((((uint64_t)value << 32) | (win >> 32)) << s) >> 32);
    high = (uint32_t)(((((uint64_t)high << 32) | 0xFFFFFFFFull) << s) >> 32);
    lowp = (lowp & 0xFFFFFFFF00000000ull) | low;
    asm("v_lshlrev_b64 %0, %1, %0" : "+v"(lowp) : "v"(s));
    win <<= s;
    left8 -= s;
    return zero;
}

// a * b + c on 24-bit signed operands (v_mad_i32_i24: the compiler would take the
// non-negative filters' products as 64-bit multiply-adds)
__device__ __forceinline__ int32_t vmad24(int32_t a, int32_t b, int32_t c) {
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// the filter update (DsdUtils.cs:431-441) of one channel after its decision (zero:
// filter0 = -1).  `q += (y - q) >> k` is written `q = (y + (2^k - 1) q) >> k` (the
// same floor), one 24-bit multiply-add and a shift (filter0 = f0): filters 1-5 stay in [0, 2^20],
// filter6 within 2^16 (Filt / fupd above).
__device__ __forceinline__ void fupd8(Filt &f, int32_t f0) {
    const int32_t v = f.q0 + (f.q7 << 3);
    const int32_t t = f.q0 - (f.q7 << 3);
    f.byte = (f.byte << 1) | (f0 & 1);
    f.q8 += (((v ^ f0) >> 31) | 1) & ((v ^ t) >> 31);
    const int32_t x = f0 & (1 << 20);
    f.q2 = vmad24(f.q2, 63, x) >> 6;
    f.q3 = vmad24(f.q3, 15, x) >> 4;
    f.q4 = vmad24(f.q4, 15, f.q3) >> 4;
    f.q5 = vmad24(f.q5, 15, f.q4) >> 4;
    const int32_t dd = (f.q5 - f.q6) >> 4;
    f.q6 += dd;
    f.q7 = vmad24(f.q7, 7, dd) >> 3;
    f.q0 = fval(f);
}

// One workgroup = two waves = 64 stereo blocks; the waves share a 64 KiB table
// array (entry e of the block of lane pair j of wave w at (e * 64 + 2j + w) * 4: the
// address a filter value selects is one v_and_or), so two workgroups fit a CU.
__device__ __forceinline__ void dsd3_pairs(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                           uint32_t n, const uint8_t *__restrict__ blob,
                                           const int32_t *__restrict__ ptables, int32_t *__restrict__ out,
                                           uint32_t *__restrict__ status) {
    using namespace wvf;
    __shared__ int32_t pt[256 * 64];
    const uint32_t tid = threadIdx.x;
    const uint32_t wv = tid >> 6, lane = tid & 63u, ch = lane & 1u, j = lane >> 1;
    const uint32_t li = blockIdx.x * 64u + wv * 32u + j;
    const bool inl = li < n;
    const uint32_t bi = inl ? list[li] : 0u;
    const BlockDesc &d = descs[bi];
    const bool ok = inl && dsd3_ok<2>(d);
    if (inl && !ok && ch == 0u) status[bi] = ST_REDO | (1u << 16);
    const uint32_t nfr = ok ? d.nframes : 0u;
    uint32_t nmax = nfr;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off));
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    uint8_t *ptb = (uint8_t *)pt;
    const uint32_t col = (2u * j + wv) * 4u;
    const int32_t chm = -(int32_t)ch;
    {   // the block's starting row (init_ptable for its rate_i), half of it by each lane of the pair
        const int32_t *row = ptables + (uint32_t)(ok ? (d.dsd_rate_i & 255) : 0) * 256u;
        // (fully unrolled: 128 loads in flight, 512 registers and a few spills here, once per
        // block; unrolled by 8 the kernel takes 129 VGPRs and no scratch, but its frame loop
        // is scheduled differently and measured 35.1 against 34.3 ms per batch, also with
        // the allocation pinned to one wave per SIMD -- profiles/r06_dsd3_regs_ab.txt)
        for (uint32_t e = ch; e < 256u; e += 2u) *(int32_t *)(ptb + (e << 8) + col) = row[e];
    }
    __syncthreads();
    if (nmax == 0u) return;
    uint32_t left8 = ok ? 8u * d.dsd_data_len : 32u;
    Win8 src;
    src.init(blob + (ok ? d.bits_off : 0), left8);
    uint64_t low = 0u;  // (decide8p: low in the low half)
    uint32_t high = 0xFFFFFFFFu;
    uint32_t value = (uint32_t)(src.win >> 32);  // init_dsd_block_high's 4 value bytes
    src.win <<= 32;
    left8 -= 32u;
    int32_t dry = src.refill(left8);
    Filt f;
    f.q2 = d.dsd_filters[ch][0];
    f.q3 = d.dsd_filters[ch][1];
    f.q4 = d.dsd_filters[ch][2];
    f.q5 = d.dsd_filters[ch][3];
    f.q6 = d.dsd_filters[ch][4];
    f.q7 = 0;
    f.q8 = d.dsd_filters[ch][5];
    f.q0 = fval(f);
    f.byte = 0;
    int32_t *o = out + d.out_off + ch;
    int32_t crc = -1;
    for (uint32_t t = 0; t < nmax; t++) {
        const bool live = t < nfr;
        // (a refill every 2 bit pairs: every 4 after the first 64 frames handed 832 of 1,024
        // blocks back dry, profiles/r06_sched_ab.txt)
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            if ((bit & 1) == 0 && bit != 0) {
                const int32_t av = src.refill(left8);
                dry = min(dry, live ? av : 0);
            }
            const uint32_t a = ((uint32_t)f.q0 & 0xFF00u) | col;
            const int32_t pv = *(const int32_t *)(ptb + a);
            const bool eq = a == (uint32_t)qp_swap((int32_t)a);
            // channel 0's entry p0, channel 1's p1 -- or the entry channel 0 just updated when
            // both chose it
            const int32_t p0 = qp_even(pv);
            int32_t p1;
            asm("v_mov_b32_dpp %0, %1 quad_perm:[1,1,3,3] row_mask:0xf bank_mask:0xf" : "=v"(p1) : "v"(pv));
            const bool z0 = decide8p(low, high, value, src.win, left8, (uint32_t)p0 >> 16);
            const int32_t nv0 = p0 + (((z0 ? kUp : kDown) - p0) >> 8);
            p1 = eq ? nv0 : p1;
            const bool z1 = decide8p(low, high, value, src.win, left8, (uint32_t)p1 >> 16);
            const int32_t nv1 = p1 + (((z1 ? kUp : kDown) - p1) >> 8);
            *(int32_t *)(ptb + a) = (ch || eq) ? nv1 : nv0;
            int32_t f0a = z0 ? -1 : 0, f0b = z1 ? -1 : 0, f0;
            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(f0) : "v"(chm), "v"(f0b), "v"(f0a));
            fupd8(f, f0);
        }
        {
            const int32_t av = src.refill(left8);
            dry = min(dry, live ? av : 0);
        }
        // the frame's bytes, CRC (crc += 2 crc + v per value, channel 0 first), factor decay (:482-489)
        const int32_t v = f.byte & 0xFF;
        const int32_t v0 = qp_even(v), v1 = qp_odd(v);
        crc = live ? (crc * 3 + v0) * 3 + v1 : crc;
        f.q8 -= (f.q8 + 512) >> 10;
        f.q0 = fval(f);
        if (live) o[2u * t] = v;
    }
    if (!ok || ch) return;
    if (dry < 0) {
        status[bi] = ST_REDO | (64u << 16);
        return;
    }
    uint32_t st = 0;
    if (d.nframes == d.block_samples) {
        st |= ST_CRC_CHECKED;
        if (crc != d.crc) {  // (the final call's mute: decoded again on the wave kernel, as dsd3_lanes)
            status[bi] = ST_REDO | (8u << 16);
            return;
        }
    }
    status[bi] = st;
}

}  // namespace dlane

__global__ void __launch_bounds__(128) wv_dsd3_pair(const BlockDesc *__restrict__ descs,
                                                    const uint32_t *__restrict__ list, uint32_t n,
                                                    const uint8_t *__restrict__ blob,
                                                    const int32_t *__restrict__ ptables, int32_t *__restrict__ out,
                                                    uint32_t *__restrict__ status) {
    dlane::dsd3_pairs(descs, list, n, blob, ptables, out, status);
}

template <int CH>
__global__ void __launch_bounds__(64) wv_dsd3_lane(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                   uint32_t n, const uint8_t *__restrict__ blob,
                                                   const int32_t *__restrict__ ptables, int32_t *__restrict__ out,
                                                   uint32_t *__restrict__ status, uint32_t *__restrict__ mute_chunk) {
    dlane::dsd3_lanes<CH>(descs, list, n, blob, ptables, out, status, mute_chunk);
}

// mode-3 blocks [0, n) of list (mono and stereo alike: one launch per channel
// count, each lane taking only its own kind; the others are handed back)
hipError_t launch_dsd3_lane(const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                            const int32_t *ptables, int32_t *out, uint32_t *status, uint32_t *mute_chunk,
                            uint32_t n_mono, hipStream_t s) {
    if (!n) return hipSuccess;
    // list order: the stereo blocks first, then n_mono mono blocks (the host sorts them)
    const uint32_t ns = n - n_mono;
    // (WVG_DSD3_PAIR=0: stereo blocks one lane each, the round-4 kernel -- A/B)
    static const bool one_lane = getenv("WVG_DSD3_PAIR") && getenv("WVG_DSD3_PAIR")[0] == '0';
    if (ns && one_lane)
        hipLaunchKernelGGL((wv_dsd3_lane<2>), dim3((ns + 63) / 64), dim3(64), 0, s, descs, list, ns, blob, ptables, out,
                           status, mute_chunk);
    else if (ns)
        hipLaunchKernelGGL(wv_dsd3_pair, dim3((ns + 63) / 64), dim3(128), 0, s, descs, list, ns, blob, ptables, out,
                           status);
    if (n_mono)
        hipLaunchKernelGGL((wv_dsd3_lane<1>), dim3((n_mono + 63) / 64), dim3(64), 0, s, descs, list + ns, n_mono, blob,
                           ptables, out, status, mute_chunk);
    return hipGetLastError();
}

}  // namespace wvg
