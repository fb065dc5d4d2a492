// wv_wave2.h -- the "two-wave" PCM block decoder for gfx950.
//
// One workgroup (2 waves) per WavPack block:
//
//   wave 0  PARSER   get_words (WordsUtils.cs:272-511) as wave-uniform scalar
//                    code (SALU + scalar branches).  The compressed payload is
//                    staged HBM -> LDS 1 KiB at a time with coalesced dwordx4
//                    loads two slots ahead of the read pointer; residuals are
//                    packed 64 per VGPR with v_writelane and handed over through
//                    an LDS ring.
//   wave 1  RECON    decorr passes (UnpackUtils.cs:688-1240) + joint stereo +
//                    mute test + CRC (:549-664) + fixup (:1251-1404) per frame,
//                    pass state in registers (term set fixed at compile time,
//                    frame loop unrolled x8 so every history index is static),
//                    output staged in VGPRs and stored 256 B per instruction.
//
// The two waves run concurrently on different SIMDs, so the block's serial
// critical path is the entropy decode alone.  Waves synchronise through LDS
// counters (workgroup-scope release/acquire) with bounded spins.
// Semantics (chunk seams, mute granularity, CRC verdicts) are those of
// decode_pcm_block in wv_decode_core.h, which the host tests check against the
// oracle; this kernel is checked against that same oracle on the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include "wv_decode_core.h"

namespace wvg {
namespace w2 {

constexpr int RES_RING = 4096;  // residual words in flight (16 KiB)
constexpr int SLOT_DW = 256;    // one staging slot = 1 KiB
constexpr int NSLOT = 4;
constexpr uint32_t SPIN_LIMIT = 1u << 26;  // bounded waits: a bug ends the kernel, never hangs the GPU

// Performance experiments (never in the shipped build): 1 = reconstruction
// wave only drains the ring, 2 = parser wave publishes zeros without parsing.
// 3 = as 1, plus parser counters written over the block's first output ints.
#ifndef WV2_EXP
#define WV2_EXP 0
#endif
#if WV2_EXP == 3
#define WV2_PROF(x) x
#else
#define WV2_PROF(x)
#endif

struct Shared {
    uint32_t stream[NSLOT * SLOT_DW];
    int32_t res[RES_RING];
    uint32_t produced;  // words available in res (parser -> recon)
    uint32_t consumed;  // words released (recon -> parser)
    uint32_t err;       // parser outcome: 0 running/ok, DEC_BITS_ERROR, DEC_EXCEPTION, 3 timeout
    uint32_t stop;      // recon asks the parser to stop (block muted)
};

__device__ __forceinline__ uint32_t lds_load_acq(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// v_writelane_b32 (lane select through M0): put a wave-uniform value into one
// lane of a VGPR.  clang has no builtin for it; this binds the LLVM intrinsic.
extern "C" __device__ int32_t wv2_writelane_i32(int32_t val, int32_t lane, int32_t old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ int32_t writelane(int32_t val, int lane_sel, int32_t vreg) {
    return wv2_writelane_i32(val, lane_sel, vreg);
}

// ---------------------------------------------------------------------------
// LDS-staged, wave-uniform bit reader with the BitReader interface used by
// get_word (64-bit window, past-the-end bytes read as 0xFF).
// ---------------------------------------------------------------------------
struct LdsReader {
    const uint8_t *blob;
    uint64_t A;  // 16-byte aligned start of the staged byte range
    uint64_t E;  // end of the real bytes
    uint32_t *ring;
    uint64_t win;
    int nb;
    uint32_t rd;      // next dword index (relative to A) to enter the window
    uint32_t nextv;   // dword rd as loaded from LDS (VGPR; read lane 0 only when it is needed)
    uint4 stage;      // chunk in flight (per lane 16 B)
    int lane;
    WV2_PROF(uint32_t n_fast = 0; uint32_t n_zr = 0; uint32_t n_slow = 0; uint32_t n_refill = 0; uint64_t t_wait = 0;)

    // Branch-free on purpose: a divergent branch anywhere in the parser makes
    // the compiler move the (uniform) bit window into VGPRs.
    __device__ __forceinline__ uint4 load_chunk(uint32_t c) const {
        uint64_t a = A + (uint64_t)c * (SLOT_DW * 4) + (uint64_t)lane * 16;
        const bool in = a < E;
        const uint4 v = *(const uint4 *)(blob + (in ? a : A));  // A is always a valid address
        const int64_t keep = in ? (int64_t)(E - a) : 0;          // real bytes in this 16 B
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int64_t kb = keep - 4 * k;
            uint32_t sh8 = (uint32_t)(kb < 0 ? 0 : (kb > 4 ? 4 : kb)) * 8;
            uint32_t m = sh8 >= 32 ? 0u : (0xFFFFFFFFu << sh8);  // bytes past the end read 0xFF
            w[k] |= m;
        }
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
    __device__ __forceinline__ void put_chunk(uint32_t c, uint4 v) {
        *(uint4 *)&ring[(c & (NSLOT - 1)) * SLOT_DW + lane * 4] = v;
    }
    __device__ __forceinline__ uint32_t lds_dw(uint32_t i) const { return uni(ring[i & (NSLOT * SLOT_DW - 1)]); }

    __device__ __forceinline__ void init(const uint8_t *b, uint64_t off, uint64_t len, uint32_t *r, int ln) {
        blob = b;
        A = off & ~(uint64_t)15;
        E = off + len;
        ring = r;
        lane = ln;
        put_chunk(0, load_chunk(0));
        put_chunk(1, load_chunk(1));
        stage = load_chunk(2);
        int skip = (int)(off - A) * 8;  // 0..120 bits
        win = (uint64_t)lds_dw(0) | ((uint64_t)lds_dw(1) << 32);
        nb = 64;
        rd = 2;
        nextv = ring[2];
        while (skip >= 32) {
            win >>= 32;
            nb -= 32;
            skip -= 32;
            refill32();
        }
        if (skip) {
            win >>= skip;
            nb -= skip;
        }
    }
    __device__ __forceinline__ void refill32() {
        win |= (uint64_t)uni(nextv) << nb;
        nb += 32;
        rd++;
        if ((rd & (SLOT_DW - 1)) == 0) {  // entering chunk c = rd / 256
            uint32_t c = rd / SLOT_DW;
            put_chunk(c + 1, stage);
            stage = load_chunk(c + 2);
        }
        nextv = ring[rd & (NSLOT * SLOT_DW - 1)];  // waited for at the next refill, not here
    }
    // 32-bit refills keep the window invariant: bits at and above nb are 0,
    // so a refill is only legal while nb <= 32; every caller needs <= 32 bits.
    __device__ __forceinline__ void need(int n) {
        if (nb < n) refill32();
    }
    __device__ __forceinline__ void skip(int n) {
        win >>= n;
        nb -= n;
    }
    __device__ __forceinline__ int getbit() {
        need(1);
        int b = (int)(win & 1);
        skip(1);
        return b;
    }
    __device__ __forceinline__ uint32_t getbits(int n) {
        if (n <= 0) return 0;
        need(n);
        uint32_t v = (uint32_t)(win & ((1ull << n) - 1));
        skip(n);
        return v;
    }
    __device__ __forceinline__ int consume_ones(int cap) {
        int total = 0;
        for (;;) {
            if (nb <= 32) refill32();  // nb in [33, 64]
            uint64_t inv = ~win;       // ones above nb stop the count at nb
            int r = inv ? __builtin_ctzll(inv) : 64;
            if (total + r >= cap) {
                skip(cap - total);
                return cap;
            }
            if (r < nb) {
                skip(r + 1);
                return total + r;
            }
            total += nb;  // the whole window was ones
            win = 0;
            nb = 0;
        }
    }
};

// ---------------------------------------------------------------------------
// parser wave.  Everything here must stay wave-uniform (SGPRs, scalar
// branches): channel indices are compile-time constants so the entropy state
// is never indexed at run time (that would put it in scratch), and no uniform
// boolean is turned into an integer (that lowers to v_cndmask and drags the
// whole loop onto the VALU).
// ---------------------------------------------------------------------------

// One residual of a lossless block, common case only (WordsUtils.cs:355-503
// with no hybrid terms): not in zero-run mode (the caller checks), fewer than
// 16 unary ones, a non-negative median, and the whole word inside the bit
// window (nb >= 32 on entry; the bound checked is unary + bitcount + 1).
// Returns false with no state changed when the word is not of that form; the
// caller then runs the general get_word.
//
// Hand-scheduled scalar code: this is the serial critical path of a block
// (one wave issues one instruction per ~4 cycles, a taken branch costs ~19),
// and the compiler's version spent ~2.5x the instructions on register
// shuffles and structurised control flow.  The bit window is copied to VCC so
// its low dword can be named (vcc_lo).  Arithmetic is exact modulo 2^32,
// which is all the output keeps: maxcode is median_k >> 4 (high - low in
// get_word), and low/mid wrap like the int64 values truncated by the (int)
// cast at WordsUtils.cs:499-503.
//   case 0:  low = 0,              mk = m0;  m0 -= ((m0+126)>>7)*2
//   case 1:  low = A0,             mk = m1;  m0 += ((m0+128)>>7)*5, m1 -= ((m1+62)>>6)*2
//   case 2:  low = A0+A1,          mk = m2;  m0, m1 += ..., m2 -= ((m2+30)>>5)*2
//   case n:  low = A0+A1+(n-2)*A2, mk = m2;  m0, m1, m2 += ...       (Ak = (mk>>4)+1)
//   read_code: n1 = bitcount-1, extras = 2^bitcount - mc - 1 (WordsUtils.cs:546-570)
#define WV2_BOUND(MK)                                   \
    "s_lshr_b32 %[mc], " MK ", 4\n"                      \
    "s_or_b32 %[t0], %[mc], 1\n"                          \
    "s_flbit_i32_b32 %[t0], %[t0]\n"                      \
    "s_sub_u32 %[n1], 31, %[t0]\n"                        \
    "s_add_u32 %[t0], %[n1], 2\n"                         \
    "s_cmp_gt_u32 %[t0], %[avail]\n"                      \
    "s_cbranch_scc1 L_done_%=\n"
#define WV2_INC(M, ADD, SH)                               \
    "s_add_i32 %[t0], " M ", " ADD "\n"                   \
    "s_ashr_i32 %[t0], %[t0], " SH "\n"                   \
    "s_mul_i32 %[t0], %[t0], 5\n"                         \
    "s_add_i32 " M ", " M ", %[t0]\n"
#define WV2_DEC(M, ADD, SH1)                              \
    "s_add_i32 %[t0], " M ", " ADD "\n"                   \
    "s_ashr_i32 %[t0], %[t0], " SH1 "\n"                  \
    "s_and_b32 %[t0], %[t0], -2\n"                        \
    "s_sub_i32 " M ", " M ", %[t0]\n"

template <int C>
__device__ __forceinline__ bool fast_word(Entropy &w, LdsReader &rd, int32_t &out) {
    uint32_t ok, o, t0, u, ones, c1, nh0, nh1, mc, n1, low, avail, ex, v;
    uint32_t nb = (uint32_t)rd.nb;
    int32_t m0 = w.med[C][0], m1 = w.med[C][1], m2 = w.med[C][2], h0 = w.h0, h1 = w.h1;
    asm volatile(
        "s_mov_b32 %[ok], 0\n"
        "s_mov_b64 vcc, %[win]\n"
        "s_cmp_lg_u32 %[h0], 0\n"
        "s_cbranch_scc1 L_h0_%=\n"
        // unary run (WordsUtils.cs:361-409 without the escape)
        "s_orn2_b32 %[t0], 0x10000, vcc_lo\n"
        "s_ff1_i32_b32 %[u], %[t0]\n"
        "s_cmp_gt_u32 %[u], 15\n"
        "s_cbranch_scc1 L_done_%=\n"
        "s_add_u32 %[c1], %[u], 1\n"
        "s_lshr_b32 %[ones], %[u], 1\n"
        "s_add_u32 %[ones], %[ones], %[h1]\n"
        "s_and_b32 %[nh1], %[u], 1\n"
        "s_xor_b32 %[nh0], %[nh1], 1\n"
        "s_sub_u32 %[avail], %[nb], %[c1]\n"
        "s_cmp_lg_u32 %[ones], 0\n"
        "s_cbranch_scc1 L_ge1_%=\n"
        "L_c0_%=:\n"
        "s_cmp_lt_i32 %[m0], 0\n"
        "s_cbranch_scc1 L_done_%=\n"
        WV2_BOUND("%[m0]")
        "s_mov_b32 %[low], 0\n"
        WV2_DEC("%[m0]", "126", "6")
        "L_tail_%=:\n"
        "s_mov_b32 %[h0], %[nh0]\n"
        "s_mov_b32 %[h1], %[nh1]\n"
        "s_lshr_b64 vcc, vcc, %[c1]\n"
        "s_sub_u32 %[nb], %[nb], %[c1]\n"
        "s_lshl_b32 %[ex], 2, %[n1]\n"
        "s_not_b32 %[t0], %[mc]\n"
        "s_add_u32 %[ex], %[ex], %[t0]\n"
        "s_bfm_b32 %[t0], %[n1], 0\n"
        "s_and_b32 %[v], vcc_lo, %[t0]\n"
        "s_cmp_lt_u32 %[v], %[ex]\n"
        "s_cbranch_scc1 L_small_%=\n"
        "s_lshr_b32 %[t0], vcc_lo, %[n1]\n"
        "s_and_b32 %[t0], %[t0], 1\n"
        "s_lshl_b32 %[v], %[v], 1\n"
        "s_sub_u32 %[v], %[v], %[ex]\n"
        "s_add_u32 %[v], %[v], %[t0]\n"
        "s_add_u32 %[n1], %[n1], 1\n"
        "L_small_%=:\n"
        "s_add_u32 %[v], %[v], %[low]\n"
        "s_lshr_b32 %[t0], vcc_lo, %[n1]\n"
        "s_bfe_i32 %[t0], %[t0], 0x10000\n"
        "s_xor_b32 %[o], %[v], %[t0]\n"
        "s_add_u32 %[n1], %[n1], 1\n"
        "s_lshr_b64 %[win], vcc, %[n1]\n"
        "s_sub_u32 %[nb], %[nb], %[n1]\n"
        "s_mov_b32 %[ok], 1\n"
        "s_branch L_done_%=\n"
        // holding_zero set: this word's unary count is 0, h1 unchanged
        "L_h0_%=:\n"
        "s_mov_b32 %[c1], 0\n"
        "s_mov_b32 %[nh0], 0\n"
        "s_mov_b32 %[nh1], %[h1]\n"
        "s_mov_b32 %[avail], %[nb]\n"
        "s_branch L_c0_%=\n"
        "L_ge1_%=:\n"
        "s_cmp_eq_u32 %[ones], 1\n"
        "s_cbranch_scc0 L_ge2_%=\n"
        "s_cmp_lt_i32 %[m1], 0\n"
        "s_cbranch_scc1 L_done_%=\n"
        WV2_BOUND("%[m1]")
        "s_ashr_i32 %[low], %[m0], 4\n"
        "s_add_u32 %[low], %[low], 1\n"
        WV2_INC("%[m0]", "128", "7")
        WV2_DEC("%[m1]", "62", "5")
        "s_branch L_tail_%=\n"
        "L_ge2_%=:\n"
        "s_cmp_lt_i32 %[m2], 0\n"
        "s_cbranch_scc1 L_done_%=\n"
        WV2_BOUND("%[m2]")
        "s_ashr_i32 %[low], %[m0], 4\n"
        "s_ashr_i32 %[t0], %[m1], 4\n"
        "s_add_u32 %[low], %[low], %[t0]\n"
        "s_add_u32 %[low], %[low], 2\n"
        WV2_INC("%[m0]", "128", "7")
        WV2_INC("%[m1]", "64", "6")
        "s_cmp_eq_u32 %[ones], 2\n"
        "s_cbranch_scc0 L_ge3_%=\n"
        WV2_DEC("%[m2]", "30", "4")
        "s_branch L_tail_%=\n"
        "L_ge3_%=:\n"
        "s_add_u32 %[t0], %[mc], 1\n"
        "s_sub_u32 %[u], %[ones], 2\n"
        "s_mul_i32 %[t0], %[t0], %[u]\n"
        "s_add_u32 %[low], %[low], %[t0]\n"
        WV2_INC("%[m2]", "32", "5")
        "s_branch L_tail_%=\n"
        "L_done_%=:\n"
        : [ok] "=&s"(ok), [o] "=&s"(o), [t0] "=&s"(t0), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1),
          [nh0] "=&s"(nh0), [nh1] "=&s"(nh1), [mc] "=&s"(mc), [n1] "=&s"(n1), [low] "=&s"(low),
          [avail] "=&s"(avail), [ex] "=&s"(ex), [v] "=&s"(v), [win] "+s"(rd.win), [nb] "+s"(nb),
          [m0] "+s"(m0), [m1] "+s"(m1), [m2] "+s"(m2), [h0] "+s"(h0), [h1] "+s"(h1)
        :
        : "vcc", "scc");
    w.med[C][0] = m0;
    w.med[C][1] = m1;
    w.med[C][2] = m2;
    w.h0 = h0;
    w.h1 = h1;
    rd.nb = (int)nb;
    out = (int32_t)o;
    return ok != 0;
}
#undef WV2_BOUND
#undef WV2_INC
#undef WV2_DEC

// one residual: the fast path for lossless blocks, the zero-run countdown,
// else the general get_word (wv_decode_core.h)
template <int C, bool LOSSLESS>
__device__ __forceinline__ int parse_word(Entropy &w, LdsReader &rd, uint32_t flags, int32_t &v) {
    if (LOSSLESS) {
        const uint32_t m00 = (uint32_t)(w.med[0][0] | w.med[1][0]);
        const bool zr = __builtin_expect(m00 <= 1u, 0) && (w.h0 | w.h1) == 0;
        if (__builtin_expect(!zr, 1)) {
            if (__builtin_expect(rd.nb < 32, 0)) rd.refill32();
            if (__builtin_expect(fast_word<C>(w, rd, v), 1)) {
                WV2_PROF(rd.n_fast++;)
                return DEC_OK;
            }
        } else if (w.zeros_acc > 1) {  // inside a zero run (WordsUtils.cs:306-311; slow_level is dead here)
            w.zeros_acc--;
            v = 0;
            WV2_PROF(rd.n_zr++;)
            return DEC_OK;
        }
    }
    WV2_PROF(rd.n_slow++;)
    return get_word(w, rd, flags, C, C == 0, v);
}

template <bool MONO, bool LOSSLESS>
__device__ __forceinline__ void parse_loop(const BlockDesc &d, LdsReader &rd, Entropy &w, Shared &sh, int lane) {
    const uint32_t flags = d.flags;
    const uint32_t total = MONO ? d.nframes : 2u * d.nframes;
    int32_t resv = 0;
    uint32_t k = 0;
    uint32_t err = 0;
    uint32_t consumed = 0;
    while (k < total) {
        const uint32_t kend = min(total, (k & ~63u) + 64u);  // next batch boundary
        while (k < kend) {
            int32_t v = 0;
            int rc = WV2_EXP == 2 ? DEC_OK : parse_word<0, LOSSLESS>(w, rd, flags, v);
            if (__builtin_expect(rc != DEC_OK, 0)) {
                err = (uint32_t)rc;
                break;
            }
            resv = writelane(v, (int)(k & 63), resv);
            k++;
            if (!MONO) {
                rc = WV2_EXP == 2 ? DEC_OK : parse_word<1, LOSSLESS>(w, rd, flags, v);
                if (__builtin_expect(rc != DEC_OK, 0)) {
                    err = (uint32_t)rc;
                    break;
                }
                resv = writelane(v, (int)(k & 63), resv);
                k++;
            }
        }
        if (err) break;
        {
            // wait for ring space, publish the batch
            uint32_t base = (k - 1) & ~63u;
            uint32_t spins = 0;
            WV2_PROF(uint64_t tw0 = clock64();)
            while (base + 64 - consumed > (uint32_t)RES_RING) {
                __builtin_amdgcn_s_sleep(2);
                consumed = uni(lds_load_acq(&sh.consumed));
                if (uni(lds_load_acq(&sh.stop))) return;  // the block was muted
                if (++spins > SPIN_LIMIT) {
                    err = 3;
                    break;
                }
            }
            WV2_PROF(rd.t_wait += clock64() - tw0;)
            if (err) break;
            sh.res[(base % RES_RING) + lane] = resv;
            lds_store_rel(&sh.produced, k);
            if (uni(lds_load_acq(&sh.stop))) return;
        }
    }
    if (err) {
        // publish the complete words before the error, then the outcome
        uint32_t base = k & ~63u;
        if ((k & 63) && err != 3) {
            uint32_t spins = 0;
            while (base + 64 - consumed > (uint32_t)RES_RING && ++spins < SPIN_LIMIT) {
                __builtin_amdgcn_s_sleep(2);
                consumed = uni(lds_load_acq(&sh.consumed));
                if (uni(lds_load_acq(&sh.stop))) return;
            }
            sh.res[(base % RES_RING) + lane] = resv;
        }
        lds_store_rel(&sh.produced, k);
        lds_store_rel(&sh.err, err);
    }
}

__device__ __forceinline__ void parser(const BlockDesc &d, const uint8_t *blob, Shared &sh, int lane, int32_t *dbg) {
    WV2_PROF(const uint64_t t_start = clock64();)
    LdsReader rd;
    rd.init(blob, d.bits_off, d.bits_len, sh.stream, lane);
    Entropy w;
#pragma unroll
    for (int c = 0; c < 2; c++) {
#pragma unroll
        for (int k = 0; k < 3; k++) w.med[c][k] = d.median[c][k];
        w.slow[c] = d.slow_level[c];
        w.errlim[c] = 0;
        w.acc[c] = d.bitrate_acc[c];
        w.dlt[c] = d.bitrate_delta[c];
    }
    w.zeros_acc = 0;
    w.h0 = w.h1 = 0;
    const bool mono = (d.flags & wvf::MONO_DATA) != 0, lossless = (d.flags & wvf::HYBRID_FLAG) == 0;
    if (mono) {
        if (lossless) parse_loop<true, true>(d, rd, w, sh, lane);
        else parse_loop<true, false>(d, rd, w, sh, lane);
    } else {
        if (lossless) parse_loop<false, true>(d, rd, w, sh, lane);
        else parse_loop<false, false>(d, rd, w, sh, lane);
    }
#if WV2_EXP == 3
    const uint64_t t_total = clock64() - t_start;
    uint32_t vals[8] = {rd.n_fast, rd.n_zr, rd.n_slow, rd.n_refill, (uint32_t)t_total, (uint32_t)(t_total >> 32),
                        (uint32_t)rd.t_wait, (uint32_t)(rd.t_wait >> 32)};
    if (lane < 8) {
        uint32_t x = vals[0];
#pragma unroll
        for (int i = 1; i < 8; i++) x = lane == i ? vals[i] : x;
        dbg[lane] = (int32_t)x;
    }
#else
    (void)dbg;
#endif
}

// ---------------------------------------------------------------------------
// reconstruction wave: pass state for a compile-time term list
// ---------------------------------------------------------------------------
template <int T>
struct PState {
    int32_t wA, wB;
    int32_t a[(T >= 17) ? 2 : 8];  // s0,s1 (17,18), ring (1..8, and mono negative), s0 (stereo negative)
    int32_t b[(T >= 17) ? 2 : 8];
    int32_t delta;

    __device__ __forceinline__ void init(const BlockDesc &d, int p) {
        wA = d.weight_A[p];
        wB = d.weight_B[p];
        delta = d.delta[p];
        if (T <= 8) {
            constexpr int TT = (T >= 1) ? T : ((T & 7) == 0 ? 8 : (T & 7));  // ring length in use
#pragma unroll
            for (int i = 0; i < 8; i++) a[i] = b[i] = 0;
            if (T >= 1 || true) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    if (i < TT) {
                        a[(8 - TT + i) & 7] = d.samples_A[p][i];
                        b[(8 - TT + i) & 7] = d.samples_B[p][i];
                    }
                }
            }
            if (T < 0) {  // stereo negative terms use slot 0 only
                a[0] = d.samples_A[p][0];
                b[0] = d.samples_B[p][0];
            }
        } else {
            a[0] = d.samples_A[p][0];
            a[1] = d.samples_A[p][1];
            b[0] = d.samples_B[p][0];
            b[1] = d.samples_B[p][1];
        }
    }
    __device__ __forceinline__ void trunc() {
        wA = (int16_t)wA;
        wB = (int16_t)wB;
    }
    // stereo frame at ring phase U (= block frame & 7)
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &L, int32_t &R) {
        using namespace wvf;
        if constexpr (T == 17 || T == 18) {
            int32_t sa = T == 17 ? sub32(mul32(2, a[0]), a[1]) : (sub32(mul32(3, a[0]), a[1]) >> 1);
            int32_t oa = add32(apply_weight(wA, sa), L);
            upd_w(wA, sa, L, delta);
            a[1] = a[0];
            a[0] = oa;
            L = oa;
            int32_t sb = T == 17 ? sub32(mul32(2, b[0]), b[1]) : (sub32(mul32(3, b[0]), b[1]) >> 1);
            int32_t ob = add32(apply_weight(wB, sb), R);
            upd_w(wB, sb, R, delta);
            b[1] = b[0];
            b[0] = ob;
            R = ob;
        } else if constexpr (T >= 1 && T <= 8) {
            int32_t sa = a[(U - T) & 7];
            int32_t oa = add32(apply_weight(wA, sa), L);
            upd_w(wA, sa, L, delta);
            a[U & 7] = oa;
            L = oa;
            int32_t sb = b[(U - T) & 7];
            int32_t ob = add32(apply_weight(wB, sb), R);
            upd_w(wB, sb, R, delta);
            b[U & 7] = ob;
            R = ob;
        } else if constexpr (T == -1) {
            int32_t sa = add32(L, apply_weight(wA, a[0]));
            upd_wc(wA, a[0], L, delta);
            int32_t o = add32(R, apply_weight(wB, sa));
            upd_wc(wB, sa, R, delta);
            L = sa;
            R = o;
            a[0] = o;
        } else if constexpr (T == -2) {
            int32_t sb = add32(R, apply_weight(wB, b[0]));
            upd_wc(wB, b[0], R, delta);
            int32_t o = add32(L, apply_weight(wA, sb));
            upd_wc(wA, sb, L, delta);
            R = sb;
            L = o;
            b[0] = o;
        } else if constexpr (T == -3) {
            int32_t sa = add32(L, apply_weight(wA, a[0]));
            upd_wc(wA, a[0], L, delta);
            int32_t sb = add32(R, apply_weight(wB, b[0]));
            upd_wc(wB, b[0], R, delta);
            b[0] = sa;
            a[0] = sb;
            L = sa;
            R = sb;
        }
    }
    template <int U>
    __device__ __forceinline__ void mono(int32_t &X) {
        using namespace wvf;
        if constexpr (T == 17 || T == 18) {
            int32_t sa = T == 17 ? sub32(mul32(2, a[0]), a[1]) : (sub32(mul32(3, a[0]), a[1]) >> 1);
            int32_t o = add32(apply_weight(wA, sa), X);
            upd_w(wA, sa, X, delta);
            a[1] = a[0];
            a[0] = o;
            X = o;
        } else {
            constexpr int TT = (T >= 1 && T <= 8) ? T : (T & 7);  // mono negative terms: default case
            int32_t sa = a[(U - (TT == 0 ? 8 : TT)) & 7];
            int32_t o = add32(apply_weight(wA, sa), X);
            upd_w(wA, sa, X, delta);
            a[U & 7] = o;
            X = o;
        }
    }
};

template <int... Ts>
struct Chain;
template <>
struct Chain<> {
    __device__ __forceinline__ void init(const BlockDesc &, int) {}
    __device__ __forceinline__ void trunc() {}
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &, int32_t &) {}
    template <int U>
    __device__ __forceinline__ void mono(int32_t &) {}
};
template <int T, int... Ts>
struct Chain<T, Ts...> {
    PState<T> p;
    Chain<Ts...> rest;
    __device__ __forceinline__ void init(const BlockDesc &d, int i) {
        p.init(d, i);
        rest.init(d, i + 1);
    }
    __device__ __forceinline__ void trunc() {
        p.trunc();
        rest.trunc();
    }
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &L, int32_t &R) {
        p.template stereo<U>(L, R);
        rest.template stereo<U>(L, R);
    }
    template <int U>
    __device__ __forceinline__ void mono(int32_t &X) {
        p.template mono<U>(X);
        rest.template mono<U>(X);
    }
};

__device__ __forceinline__ int32_t iabs(int32_t x) { return x < 0 ? (int32_t)(0u - (uint32_t)x) : x; }

// Output of the mute path: the whole chunk becomes fixup(0) and every later
// chunk 0 (UnpackUtils.cs:527-543, 649-664).  All lanes store.
template <int OCH>
__device__ __forceinline__ void mute_fill(uint32_t first_chunk, uint32_t chunk, uint32_t nfr, int32_t z0, int32_t z1,
                                          int32_t *out, uint32_t chunk_start, int lane) {
    uint32_t chunk_end = chunk_start + (chunk_start == 0 ? first_chunk : chunk);
    if (chunk_end > nfr) chunk_end = nfr;
    uint64_t a0 = (uint64_t)chunk_start * OCH, a1 = (uint64_t)chunk_end * OCH, a2 = (uint64_t)nfr * OCH;
    for (uint64_t i = a0 + lane; i < a2; i += 64) {
        int32_t v = 0;
        if (i < a1) v = (OCH == 1) ? z0 : (((i & 1) == 0) ? z0 : z1);
        out[i] = v;
    }
}

// LAYOUT 0: stereo; 1: mono (MONO_FLAG); 2: FALSE_STEREO (mono decode, 2 ints/frame)
template <int LAYOUT, int... Ts>
__device__ __forceinline__ void recon_impl(const BlockDesc &d, Shared &sh, int32_t *out_base, uint32_t *status_out,
                                           int lane) {
    using namespace wvf;
    constexpr bool MONO = LAYOUT != 0;  // mono decode path (MONO_DATA)
    constexpr int WPF = MONO ? 1 : 2;   // residual words per frame
    constexpr int OCH = LAYOUT == 1 ? 1 : 2;
    constexpr uint32_t BF = 64 / WPF;  // frames per residual batch
    const uint32_t flags = d.flags;
    const bool joint = (flags & JOINT_STEREO) != 0;
    const int32_t ml = d.mute_limit;
    const uint32_t nfr = d.nframes;
    const uint32_t chunk = d.chunk;
    int32_t *out = out_base + d.out_off;

    Chain<Ts...> ch;
    ch.init(d, 0);
    Fixup fx;
    fixup_init(fx, d);

    uint32_t status = 0;
    int32_t crc = -1;
    bool crc_garbage = false;
    uint32_t chunk_start = 0;
    uint32_t chunk_end = d.first_chunk < nfr ? d.first_chunk : nfr;
    uint32_t seam8 = (!MONO && chunk_end - chunk_start >= 16) ? chunk_start + 7 : 0xFFFFFFFFu;
    uint32_t bsp = d.first_bsp;
    bool crc_stop = false;
    uint32_t produced = 0;

    for (uint32_t t0 = 0; t0 < nfr; t0 += BF) {
        uint32_t tend = t0 + BF < nfr ? t0 + BF : nfr;
        uint32_t need = tend * WPF;
        uint32_t spins = 0;
        uint32_t perr = 0;
        while (produced < need) {
            produced = uni(lds_load_acq(&sh.produced));
            if (produced >= need) break;
            perr = uni(lds_load_acq(&sh.err));
            if (perr) {
                produced = uni(lds_load_acq(&sh.produced));
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            if (++spins > SPIN_LIMIT) {
                perr = 3;
                break;
            }
        }
        if (perr == DEC_EXCEPTION || perr == 3) {
            status |= ST_EXCEPTION;
            lds_store_rel(&sh.stop, 1);
            break;
        }
        uint32_t tvalid = produced < need ? produced / WPF : tend;  // a bits error cuts the batch short
        int32_t v = sh.res[((t0 * WPF) % RES_RING) + lane];
        int32_t o0 = 0, o1 = 0;  // staged outputs (o1: false-stereo second half)
        int mute_at = -1;

#define WV2_FRAME(U)                                                                          \
    {                                                                                         \
        const uint32_t j = g * 8 + (U);                                                       \
        const uint32_t t = t0 + j;                                                            \
        if (t < tvalid) {                                                                     \
            int32_t L, R = 0;                                                                 \
            if (MONO) {                                                                       \
                L = __builtin_amdgcn_readlane(v, (int)j);                                     \
                ch.template mono<U>(L);                                                       \
                if (!crc_stop && iabs(L) > ml) {                                              \
                    uint32_t q = bsp + (t - chunk_start);                                     \
                    if (q != chunk_end - chunk_start) {                                       \
                        mute_at = (int)t;                                                     \
                        break;                                                                \
                    }                                                                         \
                    crc_stop = true;                                                          \
                }                                                                             \
                if (!crc_stop) crc = add32(mul32(crc, 3), L);                                 \
            } else {                                                                          \
                L = __builtin_amdgcn_readlane(v, (int)(2 * j));                               \
                R = __builtin_amdgcn_readlane(v, (int)(2 * j + 1));                           \
                ch.template stereo<U>(L, R);                                                  \
                if (joint) {                                                                  \
                    R = sub32(R, L >> 1);                                                     \
                    L = add32(L, R);                                                          \
                }                                                                             \
                if (iabs(L) > ml || iabs(R) > ml) {                                           \
                    mute_at = (int)t;                                                         \
                    break;                                                                    \
                }                                                                             \
                crc = add32(mul32(add32(mul32(crc, 3), L), 3), R);                            \
            }                                                                                 \
            if (t == seam8 || t == chunk_end - 1) ch.trunc();                                 \
            const int32_t fl = fixup_tail(fx, L);                                             \
            if (LAYOUT == 1) {                                                                \
                o0 = writelane(fl, (int)j, o0);                                               \
            } else if (LAYOUT == 2) {                                                         \
                if (j < 32) {                                                                 \
                    o0 = writelane(fl, (int)(2 * j), o0);                                     \
                    o0 = writelane(fl, (int)(2 * j + 1), o0);                                 \
                } else {                                                                      \
                    o1 = writelane(fl, (int)(2 * j - 64), o1);                                \
                    o1 = writelane(fl, (int)(2 * j - 63), o1);                                \
                }                                                                             \
            } else {                                                                          \
                o0 = writelane(fl, (int)(2 * j), o0);                                         \
                o0 = writelane(fixup_tail(fx, R), (int)(2 * j + 1), o0);                      \
            }                                                                                 \
            if (t == chunk_end - 1) {                                                         \
                chunk_start = t + 1;                                                          \
                chunk_end = chunk_start + chunk < nfr ? chunk_start + chunk : nfr;            \
                seam8 = (!MONO && chunk_end - chunk_start >= 16) ? chunk_start + 7 : 0xFFFFFFFFu; \
                bsp = 0;                                                                      \
                crc_stop = false;                                                             \
            }                                                                                 \
        }                                                                                     \
    }

        for (uint32_t g = 0; g < BF / 8; g++) {
            if (WV2_EXP == 1 || WV2_EXP == 3 || t0 + g * 8 >= tvalid) break;
            do {
                WV2_FRAME(0) WV2_FRAME(1) WV2_FRAME(2) WV2_FRAME(3) WV2_FRAME(4) WV2_FRAME(5) WV2_FRAME(6) WV2_FRAME(7)
            } while (0);
            if (mute_at >= 0) break;
        }
#undef WV2_FRAME
        // store the batch: 64 ints per instruction, one per lane
        const uint32_t nv = (mute_at >= 0 ? (uint32_t)mute_at : tvalid) - t0;
        const uint64_t base = (uint64_t)t0 * OCH;
        if (WV2_EXP != 3 && (uint32_t)lane < nv * OCH) out[base + lane] = o0;
        if (LAYOUT == 2 && (uint32_t)lane + 64 < nv * OCH) out[base + 64 + lane] = o1;
        const bool bits_err = tvalid < tend;
        if (mute_at >= 0 || bits_err) {
            if (bits_err && mute_at < 0) {
                status |= ST_BITS_ERROR;
                crc_garbage = true;
                if (MONO && chunk_start == 0 && bsp > 0) status |= ST_NONDET;
            }
            status |= ST_MUTED;
            lds_store_rel(&sh.stop, 1);
            const int32_t z0 = fixup_tail(fx, 0);
            mute_fill<OCH>(d.first_chunk, chunk, nfr, z0, z0, out, chunk_start, lane);
            break;
        }
        lds_store_rel(&sh.consumed, tend * WPF);
    }
    if (!(status & ST_EXCEPTION) && nfr == d.block_samples) {
        status |= ST_CRC_CHECKED;
        if (crc_garbage || crc != d.crc) status |= ST_CRC_ERROR;
    }
    if (lane == 0) *status_out = d.fstatus | status;
}

template <int... Ts>
__device__ __forceinline__ void recon(const BlockDesc &d, Shared &sh, int32_t *out, uint32_t *status_out, int lane) {
    const uint32_t f = d.flags;
    if (f & wvf::FALSE_STEREO)
        recon_impl<2, Ts...>(d, sh, out, status_out, lane);
    else if (f & wvf::MONO_FLAG)
        recon_impl<1, Ts...>(d, sh, out, status_out, lane);
    else
        recon_impl<0, Ts...>(d, sh, out, status_out, lane);
}

template <int... Ts>
__device__ __forceinline__ void block_2wave(const BlockDesc *descs, const uint32_t *list, const uint8_t *blob, int32_t *out,
                            uint32_t *status) {
    __shared__ Shared sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    if (threadIdx.x == 0) {
        sh.produced = 0;
        sh.consumed = 0;
        sh.err = 0;
        sh.stop = 0;
    }
    __syncthreads();
    if (wave == 0)
        parser(d, blob, sh, lane, out + d.out_off);
    else
        recon<Ts...>(d, sh, out, &status[bi], lane);
}

}  // namespace w2
}  // namespace wvg
