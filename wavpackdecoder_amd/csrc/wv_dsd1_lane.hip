// wv_dsd1_lane.hip -- DSD mode 1 (DsdUtils.init_dsd_block_fast + decode_fast,
// DsdUtils.cs:149-304) with 16 lanes per block, 4 blocks per wave: the throughput
// kernel for batches with many mode-1 blocks (the lane kernels' choice,
// wvg_batch_set_kernel(WVG_KERNEL_LANE) or WVG_KERNEL_AUTO once batches overlap).
//
// A mode-1 block is one serial range-coder chain over 8-bit symbols: per symbol
// mult = (high - low) / tot[p0], index = (value - low) / mult, the symbol is the
// entry of the bin-p0 cumulative table that index falls in, and low / high move
// to that entry's bounds.  One block's tables (history_bins x 256 probabilities,
// up to 32 x 256) do not fit in a lane's share of LDS, so here a block owns a
// 16-lane row of the wave (DPP rows are 16 lanes wide) and its tables sit in LDS
// as bytes plus per-segment running sums (9.5 KiB a block; 4 blocks a wave, 4
// waves a CU):
//   prob[b][i]   the probabilities (u8),
//   base[b][s]   summed_probabilities at the end of segment s (entries 16s..16s+15),
//   gm[b]        an invariant-divisor reciprocal of tot[b] = base[b][15] (Granlund-
//                Montgomery: mult is one mul_hi, four shifts / adds -- no division).
// Per symbol the row finds the entry without dividing by mult: lane j compares
// base[p0][j] * mult against value - low (products stay inside range: base <= tot and
// tot * mult <= high - low), so the segment is the count of lanes at or below it (a
// ballot), then lane j reads the segment's probability j, a row prefix sum (4 DPP
// steps) gives the running sums, and a second compare and count gives the entry.
// low / high move by the largest product at or below value - low and the smallest
// above it (row max / min, DPP).  Everything else -- the renormalisation, the crc,
// the history bins -- is the same per lane of the row.
//
// Exactness by hand-back: a block outside the kernel's scope (a seek's discard calls,
// state from an earlier block, a framing verdict), a symbol the reference would fail
// (an empty bin, index >= tot: its `return 0`), or a CRC mismatch at the block's end
// (the final call's 0x55 mute) is marked ST_REDO and decoded again right after by
// wv_decode_dsd_fast (one wave per block), whose results the GPU tests hold against
// the oracle.
#include <hip/hip_runtime.h>

#include "wv_desc.h"
#include "wv_format.h"

namespace wvg {
namespace d1lane {

#ifndef WV_D1_PF  // (A/B builds) the window's load consumed a refill after it is issued
#define WV_D1_PF 0
#endif
#ifndef WV_D1_PRE  // (A/B builds) stereo: the next symbol's bin read while this one decodes
#define WV_D1_PRE 0
#endif
#ifndef WV_D1_SEGLDS  // (A/B builds) the segment's start read from LDS, not a row max (slower: an LDS
#define WV_D1_SEGLDS 0  // round trip on the chain, where the row max overlaps the probability read)
#endif
#ifndef WV_D1_BPERM  // (A/B builds) low / high from lanes cnt - 1 / cnt by ds_bpermute, not row max / min
#define WV_D1_BPERM 0   // (slower: the permute's LDS latency on the chain)
#endif
#ifndef WV_D1_UFLUSH  // (A/B builds) stereo: the output staged and stored at uniform points
#define WV_D1_UFLUSH 1
#endif
constexpr uint32_t ST_REDO = 1u << 15;  // as wv_lane.h: decode this block again (wave kernel)
constexpr uint32_t kBins = 32;          // init_dsd_block_fast: history_bits <= MAX_HISTORY_BITS (5)

// one block's tables in LDS
struct Slot {
    uint8_t prob[kBins * 256];   // probabilities, bin-major
    uint16_t base[kBins * 16];   // running sum at the end of each 16-entry segment
    uint32_t gm[kBins][2];       // reciprocal of the bin's total: magic, s1 | s2 << 8
};
static_assert(sizeof(Slot) == 9472, "slot layout");

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// row (16-lane) reductions and scans over DPP
template <int CTRL, bool BOUND>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, BOUND);
}
__device__ __forceinline__ uint32_t row_max(uint32_t v) {
    v = max(v, dpp<0x121, false>(v));  // row_ror:1
    v = max(v, dpp<0x122, false>(v));  // row_ror:2
    v = max(v, dpp<0x124, false>(v));  // row_ror:4
    return max(v, dpp<0x128, false>(v));  // row_ror:8
}
__device__ __forceinline__ uint32_t row_min(uint32_t v) {
    v = min(v, dpp<0x121, false>(v));
    v = min(v, dpp<0x122, false>(v));
    v = min(v, dpp<0x124, false>(v));
    return min(v, dpp<0x128, false>(v));
}
__device__ __forceinline__ uint32_t row_scan(uint32_t v) {  // inclusive prefix sum within the row
    v += dpp<0x111, true>(v);  // row_shr:1 (lanes shifted in from outside the row read 0)
    v += dpp<0x112, true>(v);
    v += dpp<0x114, true>(v);
    return v + dpp<0x118, true>(v);
}
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {  // inclusive prefix sum over the wave
    v = row_scan(v);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}
// the number of set bits of the lane's row in a ballot mask
__device__ __forceinline__ uint32_t row_count(uint64_t m, uint32_t rsh) {
    return (uint32_t)__builtin_popcount((uint32_t)(m >> rsh) & 0xFFFFu);
}
__device__ __forceinline__ uint32_t gm_div(uint32_t mag, uint32_t sh, uint32_t n) {
    const uint32_t t1 = __umulhi(mag, n);
    return (t1 + ((n - t1) >> (sh & 0xFFu))) >> (sh >> 8);
}

// per-lane payload window: byte 0 in bits 63..56 of win, avail bytes valid (>= 4
// between symbols), q0 / q1 the two dwords after them, ld the load of the dword after
// those, issued at the previous refill: a refill consumes only a load issued a symbol
// (hundreds of cycles) earlier, so no symbol waits on memory -- a select on a load issued
// in the same refill would wait for it there (the compiler's vmcnt)
struct Win {
    const uint32_t *w;
    uint64_t win;
    int32_t avail;
    uint32_t ni, q0, q1, ld;
    __device__ __forceinline__ void init(const uint8_t *p) {
        const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
        w = (const uint32_t *)(p - sh);
        win = (uint64_t)bswap(w[0]) << (32u + 8u * sh);
        avail = 4 - (int32_t)sh;
        q0 = w[1];
        q1 = w[2];
        ld = w[3];
        ni = 3;
        refill();
    }
    __device__ __forceinline__ void refill() {  // branch-free: a lane with more than 4 bytes keeps its window
        const bool m = avail <= 4;
        const uint32_t sh = (uint32_t)(32 - 8 * (m ? avail : 0)) & 63u;
        win |= m ? (uint64_t)bswap(q0) << sh : 0ull;
        avail += m ? 4 : 0;
#if WV_D1_PF
        q0 = m ? q1 : q0;
        q1 = m ? ld : q1;
        ni += m ? 1u : 0u;
        ld = w[ni];  // (reads stay within 16 bytes past the consumed ones: the blob's 64-B tail)
#else
        const uint32_t nn = w[ni];
        q0 = m ? q1 : q0;
        q1 = m ? nn : q1;
        ni += m ? 1u : 0u;
#endif
    }
};

// can a row decode block d exactly (else ST_REDO)?  CH: channels decoded
template <int CH>
__device__ __forceinline__ bool m1_ok(const BlockDesc &d) {
    using namespace wvf;
    if (d.kind != KIND_DSD_FAST) return false;
    if (((d.flags & MONO_DATA) ? 1 : 2) != CH) return false;
    if (((CH == 2 || (d.flags & FALSE_STEREO)) ? 2u : 1u) != d.out_nch) return false;
    if (d.inherit || d.chain_len >= 2 || d.pre_end || d.fstatus) return false;
    const uint32_t bins = (uint32_t)d.dsd_history_bins;
    if (bins == 0u || bins > kBins || (bins & (bins - 1u))) return false;
    if (d.dsd_data_len < 4u) return false;
    return true;
}

// init_dsd_block_fast's tables (DsdUtils.cs:169-229) for one block, by the whole wave:
// the probabilities (run-length codes decoded 64 per step, a wave prefix sum of the
// run lengths placing each; or copied when max_probability is 0xFF), then per bin the
// segment sums (summed_probabilities at every 16th entry) and the reciprocal of the
// bin's total.  The framing ran the reference's checks on the same bytes.
__device__ __forceinline__ void build(const BlockDesc &d, const uint8_t *__restrict__ blob, Slot &S, uint32_t lane) {
    const uint32_t bins = (uint32_t)d.dsd_history_bins;
    const uint32_t ne = bins * 256u;
    uint32_t *pw = (uint32_t *)S.prob;
    const uint8_t *src = blob + d.dsd_prob_off;
    if (d.dsd_max_prob < 0xFF) {
        for (uint32_t i = lane; i < ne / 16u; i += 64) ((uint4 *)S.prob)[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        const uint32_t maxp = (uint32_t)d.dsd_max_prob;
        // codes past the terminating one are read but not used: the address stays within
        // the 4 value bytes and 63 bytes past them (payload, then the blob's 64-B tail)
        const uint32_t lim = (uint32_t)(d.bits_off - d.dsd_prob_off) + 63u;
        uint32_t outptr = 0, p = 0;
        uint32_t c = src[min(lane, lim)];
        for (;;) {
            const uint32_t cn = src[min(p + 64u + lane, lim)];  // the next step's codes, in flight meanwhile
            const uint32_t len = c > maxp ? c - maxp : (c != 0u ? 1u : 0u);
            const uint32_t incl = wave_scan(len);
            // the loop ends at the first 0 code, or once the entries are all filled
            const uint64_t ev = __ballot(c == 0u || outptr + incl >= ne);
            const uint32_t last = ev ? (uint32_t)__builtin_ctzll(ev) : 63u;
            if (lane <= last && c != 0u && c <= maxp) S.prob[outptr + incl - 1u] = (uint8_t)c;
            outptr += (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)last);
            p += last + 1u;
            if (ev) break;
            c = cn;
        }
    } else {
        const uint32_t sh = (uint32_t)(d.dsd_prob_off & 3u);
        const uint32_t *g = (const uint32_t *)(src - sh);
        for (uint32_t i = lane; i < ne / 4u; i += 64) pw[i] = __builtin_amdgcn_alignbyte(g[i + 1u], g[i], sh);
    }
    __syncthreads();
    uint32_t my_tot = 0;
    for (uint32_t b = 0; b < bins; b++) {
        const uint32_t w = pw[b * 64u + lane];
        const uint32_t s4 = (w & 0xFFu) + ((w >> 8) & 0xFFu) + ((w >> 16) & 0xFFu) + (w >> 24);
        const uint32_t incl = wave_scan(s4);  // (<= 256 x 255: summed_probabilities' ushort never wraps)
        if ((lane & 3u) == 3u) S.base[b * 16u + (lane >> 2)] = (uint16_t)incl;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        my_tot = lane == b ? tot : my_tot;
    }
    if (lane < bins) {
        // lane b: bin b's total and the constants of dividing by it (all zero for an empty
        // bin: mult is then the range itself, every product <= value - low, and the row's
        // count of 16 fails the symbol, the C#'s `return 0`)
        uint32_t mag = 0, s1 = 0, s2 = 0;
        if (my_tot) {
            const uint32_t l = my_tot > 1u ? 32u - (uint32_t)__clz(my_tot - 1u) : 0u;  // ceil(log2 tot)
            mag = (uint32_t)(((((uint64_t)1 << l) - my_tot) << 32) / my_tot) + 1u;
            s1 = l ? 1u : 0u;
            s2 = l ? l - 1u : 0u;
        }
        S.gm[lane][0] = mag;
        S.gm[lane][1] = s1 | (s2 << 8);
    }
}

// One workgroup = one wave = 4 blocks, 16 lanes each (row r of the wave: block 4w + r)
template <int CH>
__device__ __forceinline__ void m1_rows(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                       uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                       uint32_t *__restrict__ status, uint32_t *__restrict__ mute_chunk) {
    using namespace wvf;
    __shared__ Slot slots[4];
    const uint32_t lane = threadIdx.x, row = lane >> 4, j = lane & 15u, rsh = row * 16u;
    const uint32_t li = blockIdx.x * 4u + row;
    const bool inl = li < n;
    const uint32_t bi = inl ? list[li] : 0u;
    const BlockDesc &d = descs[bi];
    const bool ok = inl && m1_ok<CH>(d);
    // the tables of the wave's blocks, one block at a time by all 64 lanes
    for (uint32_t r = 0; r < 4u; r++) {
        const uint32_t lr = blockIdx.x * 4u + r;
        if (lr >= n) break;
        const BlockDesc &dr = descs[list[lr]];
        if (m1_ok<CH>(dr)) build(dr, blob, slots[r], lane);  // (a uniform test: every lane reads the same block)
    }
    __syncthreads();
    if (inl && !ok && j == 0u) status[bi] = ST_REDO | (1u << 16);
    const uint32_t nfr = ok ? d.nframes : 0u;
    uint32_t nmax = nfr;
#pragma unroll
    for (int off = 32; off >= 16; off >>= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off));
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    if (nmax == 0u) return;
    const Slot &S = slots[row];
    const uint32_t bmask = ok ? (uint32_t)d.dsd_history_bins - 1u : 0u;
    Win src;
    src.init(blob + (ok ? d.bits_off : 0));
    uint32_t left = ok ? d.dsd_data_len : 4u;
    uint32_t value = (uint32_t)(src.win >> 32);  // init_dsd_block_fast's 4 value bytes
    src.win <<= 32;
    src.avail -= 4;
    left -= 4u;
    src.refill();
    uint32_t low = 0u, high = 0xFFFFFFFFu, p0 = 0u, p1 = 0u, crc = 0xFFFFFFFFu, bad = 0u;
    int32_t dry = 0;
    // output staging: int k of the row's next 16 in lane k; a FALSE_STEREO symbol is two ints
    const uint32_t wps = (CH == 1 && (d.flags & FALSE_STEREO)) ? 2u : 1u;
    int32_t *o = out + d.out_off;
    uint32_t nst = 0u, obase = 0u;
    int32_t stg = 0;
    // a bin's reciprocal and this lane's segment end: read a symbol ahead for stereo (the
    // next symbol's bin is p1 before this one decodes: each channel's history is its own
    // previous symbol, DsdUtils.cs:290-292), after the symbol for mono (its own code)
    struct Pre {
        uint32_t mag, gsh, be;
    };
    auto pre = [&](uint32_t pa) -> Pre { return Pre{S.gm[pa][0], S.gm[pa][1], (uint32_t)S.base[pa * 16u + j]}; };
    Pre cur = pre(0u);
    auto symbol = [&](bool act) {
        const uint32_t pa = p0;
        const uint32_t mag = cur.mag, gsh = cur.gsh, be = cur.be;
        Pre nx;
        if (CH == 2 && WV_D1_PRE) nx = pre(p1);
        uint32_t mult = gm_div(mag, gsh, high - low);
        if (__builtin_expect(__ballot(act && mult == 0u) != 0ull, 0)) {
            // DsdUtils.cs:262-274: four more value bytes (when there are), the full range
            const bool z = act && mult == 0u;
            const bool take = z && left >= 4u;
            value = take ? (uint32_t)(src.win >> 32) : value;
            src.win = take ? src.win << 32 : src.win;
            src.avail -= take ? 4 : 0;
            left -= take ? 4u : 0u;
            src.refill();
            low = z ? 0u : low;
            high = z ? 0xFFFFFFFFu : high;
            mult = z ? gm_div(mag, gsh, 0xFFFFFFFFu) : mult;
        }
        const uint32_t x = value - low;
        // the segment: entries 16 seg .. 16 seg + 15 hold index = x / mult
        const uint32_t q1 = be * mult;
        const bool c1 = q1 <= x;
        const uint32_t seg = row_count(__ballot(c1), rsh);
        bad |= (act && seg >= 16u) ? 2u : 0u;  // index >= tot (or an empty bin)
        const uint32_t sg = min(seg, 15u);
#if WV_D1_SEGLDS
        // the running sum before the segment: the previous segment's end, read beside the
        // segment's probabilities
        const uint32_t segstart = seg ? (uint32_t)S.base[pa * 16u + sg - 1u] : 0u;
#else
        const uint32_t segstart = row_max(c1 ? be : 0u);  // running sum before the segment
#endif
        const uint32_t pbv = S.prob[pa * 256u + (sg << 4) + j];
        const uint32_t q2 = (segstart + row_scan(pbv)) * mult;
        const bool c2 = q2 <= x;
        const uint32_t cnt = row_count(__ballot(c2), rsh);
        const uint32_t code = (seg << 4) + cnt;
        // low += summed[code - 1] * mult; high = low + prob[code] * mult - 1 (:281-284)
#if WV_D1_BPERM
        // the products of entries code - 1 and code: lanes cnt - 1 and cnt of the row
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rsh + cnt) << 2), (int)q2);
        const uint32_t lq = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rsh + cnt - 1u) << 2), (int)q2);
        const uint32_t lo = cnt ? lq : segstart * mult;
#else
        // (entry code - 1's product is the largest at or below x: a lane of the segment, or
        // for cnt == 0 the previous segment's end, lane seg - 1's q1)
        const uint32_t lo = row_max(c2 ? q2 : (c1 ? q1 : 0u));
        const uint32_t hi = row_min(c2 ? 0xFFFFFFFFu : q2);
#endif
        // (a row past its block's end decodes on, unobserved: its reads stay inside its
        // data -- `left` -- and its table; the crc, the verdicts and the stores are gated)
        high = low + hi - 1u;
        low = low + lo;
        uint32_t c3;  // crc * 3 (full-rate; the compiler's choice is a 64-bit multiply-add)
        asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(c3) : "v"(crc));
        crc = act ? c3 + code : crc;
        if (CH == 2) {
            p0 = p1;
            p1 = code & bmask;
            if (WV_D1_PRE) cur = nx;
            else cur = pre(p0);
        } else {
            p0 = code & bmask;
            cur = pre(p0);
        }
        // the byte loop (:295-300) as one shift by the leading zero bytes of high ^ low,
        // capped by the bytes left
        uint32_t lz;
        asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(high ^ low));
        const uint32_t nb = min(min(lz >> 3, 4u), left);
        const uint32_t s = nb << 3;
        value = (uint32_t)(((((uint64_t)value << 32) | (src.win >> 32)) << s) >> 32);
        high = (uint32_t)(((((uint64_t)high << 32) | 0xFFFFFFFFull) << s) >> 32);
        low = (uint32_t)(((uint64_t)low << s) & 0xFFFFFFFFull);
        src.win <<= s;
        src.avail -= (int32_t)nb;
        left -= nb;
        dry = act ? min(dry, src.avail) : dry;
        src.refill();
        // stage the symbol's int(s); a row's 16 ints go out in one store
        if (CH == 2 && WV_D1_UFLUSH) {
            // stereo: int k of a frame run is symbol k (every row at the same position)
            stg = (act && j == nst) ? (int32_t)code : stg;
            nst = (nst + 1u) & 15u;
        } else {
            if (act) {
                stg = (j == nst || (wps == 2u && j == nst + 1u)) ? (int32_t)code : stg;
                nst += wps;
            }
            if (nst == 16u) {
                o[obase + j] = stg;
                obase += 16u;
                nst = 0u;
            }
        }
    };
    const uint32_t nint = nfr * (CH == 2 ? 2u : wps);  // the row's ints
    for (uint32_t t = 0; t < nmax; t++) {
        const bool act = t < nfr;
        symbol(act);
        if (CH == 2) {
            symbol(act);
            if (WV_D1_UFLUSH && (t & 7u) == 7u) {  // (uniform) every 8 frames: each row's 16 ints, or its last ones
                if (obase + j < nint) o[obase + j] = stg;
                obase += 16u;
            }
        }
    }
    if (CH == 2 && WV_D1_UFLUSH) {
        if (obase + j < nint) o[obase + j] = stg;
    } else if (ok && j < nst) {
        o[obase + j] = stg;
    }
    if (!ok || j != 0u) return;
    if (bad || dry < 0) {
        status[bi] = ST_REDO | ((bad ? 2u : 64u) << 16);
        return;
    }
    uint32_t st = 0;
    if (d.nframes == d.block_samples) {
        st |= ST_CRC_CHECKED;
        if ((int32_t)crc != d.crc) {
            // DsdUtils.cs:99-117: the final call mutes -- the wave kernel's call-by-call output
            status[bi] = ST_REDO | (8u << 16);
            return;
        }
    }
    status[bi] = st;
    mute_chunk[bi] = 0u;
}

}  // namespace d1lane

template <int CH>
__global__ void __launch_bounds__(64) wv_dsd1_lane(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                   uint32_t n, const uint8_t *__restrict__ blob,
                                                   int32_t *__restrict__ out, uint32_t *__restrict__ status,
                                                   uint32_t *__restrict__ mute_chunk) {
    d1lane::m1_rows<CH>(descs, list, n, blob, out, status, mute_chunk);
}

// mode-1 blocks [0, n) of list: the stereo blocks first, then n_mono mono (and mono
// false-stereo) blocks (the host sorts them); a row taking a block of the other kind
// hands it back
hipError_t launch_dsd1_lane(const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                            int32_t *out, uint32_t *status, uint32_t *mute_chunk, uint32_t n_mono, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t ns = n - n_mono;
    if (ns)
        hipLaunchKernelGGL((wv_dsd1_lane<2>), dim3((ns + 3) / 4), dim3(64), 0, s, descs, list, ns, blob, out, status,
                           mute_chunk);
    if (n_mono)
        hipLaunchKernelGGL((wv_dsd1_lane<1>), dim3((n_mono + 3) / 4), dim3(64), 0, s, descs, list + ns, n_mono, blob, out,
                           status, mute_chunk);
    return hipGetLastError();
}

}  // namespace wvg
