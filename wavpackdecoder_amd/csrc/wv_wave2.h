// wv_wave2.h -- the "two-wave" PCM block decoder for gfx950.
//
// One workgroup (2 waves) per WavPack block:
//
//   wave 0  PARSER   get_words (WordsUtils.cs:272-511) as wave-uniform scalar
//                    code (SALU + scalar branches).  The compressed payload is
//                    read through the scalar cache (s_load, a dword or two
//                    ahead of a 64-bit bit window); residuals are packed 64 per
//                    VGPR with v_writelane and handed over through an LDS ring.
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

constexpr int RES_RING = 2048;  // residual words in flight (8 KiB: 2 waves x 8 KiB lets 16 blocks share a CU)
constexpr uint32_t SPIN_LIMIT = 1u << 26;  // bounded waits: a bug ends the kernel, never hangs the GPU
// the reconstruction wave's poll interval (s_sleep units of 64 cycles): its
// polls issue scalar instructions on the SIMD the parser waves are bound on
constexpr int WV2_RECON_SLEEP = 64;
// the reconstruction wave's wait bound in polls: about the same wall time
// (~4 s) as SPIN_LIMIT polls of s_sleep 2
constexpr uint32_t RECON_SPIN_LIMIT = SPIN_LIMIT / (WV2_RECON_SLEEP > 2 ? WV2_RECON_SLEEP / 2 : 1);

// The reconstruction wave keeps the parser's payload ahead of it in the CU's
// scalar cache: a scalar load per 64-byte line up to PF_AHEAD bytes past the
// position the parser last published.
constexpr uint32_t PF_AHEAD = 1024u;

struct Shared {
    int32_t res[RES_RING];
    uint32_t produced;  // words available in res (parser -> recon)
    uint32_t consumed;  // words released (recon -> parser)
    uint32_t err;       // parser outcome: 0 running/ok, DEC_BITS_ERROR, DEC_EXCEPTION, DEC_TIMEOUT
    uint32_t stop;      // recon asks the parser to stop (block muted)
    uint32_t pos;       // parser's read position (dword index), a prefetch hint
};

__device__ __forceinline__ uint32_t lds_load_acq(uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_rel(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Publish a counter after this wave's LDS writes: DS operations of one wave
// complete in order, so waiting for the LDS queue is enough; a release store
// would also wait for every outstanding global load/store (vmcnt(0)).
__device__ __forceinline__ void lds_publish(uint32_t *p, uint32_t v) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// v_writelane_b32 (lane select through M0): put a wave-uniform value into one
// lane of a VGPR.  clang has no builtin for it; this binds the LLVM intrinsic.
extern "C" __device__ int32_t wv2_writelane_i32(int32_t val, int32_t lane, int32_t old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ int32_t writelane(int32_t val, int lane_sel, int32_t vreg) {
    return wv2_writelane_i32(val, lane_sel, vreg);
}

// ---------------------------------------------------------------------------
// Scalar-memory bit reader with the BitReader interface used by get_word:
// the payload is read dword by dword with s_load (constant address space, so
// the loads are scalar and go through the scalar cache), two dwords ahead of
// the window; bytes at or past the end read as 0xFF (BitsUtils.cs:125-139).
// No LDS staging, no VALU, no cross-lane moves on the refill path.
// ---------------------------------------------------------------------------
typedef const __attribute__((address_space(4))) uint32_t *cdw_ptr;

struct SmemReader {
    cdw_ptr base;   // dword-aligned start of the payload
    uint32_t E;     // real bytes from base
    uint64_t win;
    int nb;
    uint32_t rd;    // index of the next dword to enter the window (== n0)
    uint32_t n0, n1;

    __device__ __forceinline__ uint32_t ld(uint32_t i) const {
        const uint32_t b = 4u * i;
        if (__builtin_expect(b + 4u <= E, 1)) return base[i];
        if (b >= E) return 0xFFFFFFFFu;
        return base[i] | (0xFFFFFFFFu << (8u * (E - b)));  // partial last dword (the blob is padded)
    }
    __device__ __forceinline__ void init(const uint8_t *blob, uint64_t off, uint64_t len) {
        const uint64_t a = off & ~(uint64_t)3;
        base = (cdw_ptr)(blob + a);
        E = (uint32_t)(len + (off - a));
        win = (uint64_t)ld(0) | ((uint64_t)ld(1) << 32);
        nb = 64;
        rd = 2;
        n0 = ld(2);
        n1 = ld(3);
        const int skip = (int)(off - a) * 8;
        if (skip) {
            win >>= skip;
            nb -= skip;
        }
    }
    __device__ __forceinline__ void refill32() {
        win |= (uint64_t)n0 << nb;
        nb += 32;
        rd++;
        n0 = n1;
        n1 = ld(rd + 1);
    }
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
            if (nb <= 32) refill32();
            uint64_t inv = ~win;
            int r = inv ? __builtin_ctzll(inv) : 64;
            if (total + r >= cap) {
                skip(cap - total);
                return cap;
            }
            if (r < nb) {
                skip(r + 1);
                return total + r;
            }
            total += nb;
            win = 0;
            nb = 0;
        }
    }
};

typedef SmemReader Reader;

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
__device__ __forceinline__ bool fast_word(Entropy &w, Reader &rd, int32_t &out) {
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

// ---------------------------------------------------------------------------
// The lossless inner loop as one scalar sequence: words k..kend-1 (stereo:
// alternating channel contexts 0/1 starting at channel 0), each the common
// case of fast_word, with the bit window held in VCC (so its halves can be
// named) and the SmemReader refill (two dwords prefetched with s_load) done
// in place.  Exits early (reason 1) before touching any state of a word that
// is not of the common form, or when a refill would read near the payload
// end; the caller then runs the general get_word for that word.  Leaves no
// scalar load outstanding.
// ---------------------------------------------------------------------------
#define WV2_W_BOUND(MK)                                       \
    "s_lshr_b32 %[mc], " MK ", 4\n"                            \
    "s_or_b32 %[t0], %[mc], 1\n"                                \
    "s_flbit_i32_b32 %[t0], %[t0]\n"                            \
    "s_sub_u32 %[n1], 31, %[t0]\n"                              \
    "s_add_u32 %[t0], %[n1], 2\n"                               \
    "s_cmp_gt_u32 %[t0], %[avail]\n"                            \
    "s_cbranch_scc1 LB" C "_%=\n"
#define WV2_W_INC(M, ADD, SH)                                   \
    "s_add_i32 %[t0], " M ", " ADD "\n"                         \
    "s_ashr_i32 %[t0], %[t0], " SH "\n"                         \
    "s_mul_i32 %[t0], %[t0], 5\n"                               \
    "s_add_i32 " M ", " M ", %[t0]\n"
#define WV2_W_DEC(M, ADD, SH1)                                  \
    "s_add_i32 %[t0], " M ", " ADD "\n"                         \
    "s_ashr_i32 %[t0], %[t0], " SH1 "\n"                        \
    "s_and_b32 %[t0], %[t0], -2\n"                              \
    "s_sub_i32 " M ", " M ", %[t0]\n"
// read_code + sign + window advance + residual into lane M0 (WordsUtils.cs:494-503, 546-570)
#define WV2_TAIL(C, SFX)                                                                 \
    "s_lshr_b64 vcc, vcc, %[c1]\n"                                               \
    "s_sub_u32 %[nb], %[nb], %[c1]\n"                                            \
    "s_lshl_b32 %[ex], 2, %[n1]\n"                                               \
    "s_not_b32 %[t0], %[mc]\n"                                                   \
    "s_add_u32 %[ex], %[ex], %[t0]\n"                                            \
    "s_bfm_b32 %[t0], %[n1], 0\n"                                                \
    "s_and_b32 %[v], vcc_lo, %[t0]\n"                                            \
    "s_cmp_lt_u32 %[v], %[ex]\n"                                                 \
    "s_cbranch_scc1 LS" C SFX "_%=\n"                                            \
    "s_lshr_b32 %[t0], vcc_lo, %[n1]\n"                                          \
    "s_and_b32 %[t0], %[t0], 1\n"                                                \
    "s_lshl_b32 %[v], %[v], 1\n"                                                 \
    "s_sub_u32 %[v], %[v], %[ex]\n"                                              \
    "s_add_u32 %[v], %[v], %[t0]\n"                                              \
    "s_add_u32 %[n1], %[n1], 1\n"                                                \
    "LS" C SFX "_%=:\n"                                                          \
    "s_add_u32 %[v], %[v], %[low]\n"                                             \
    "s_lshr_b32 %[t0], vcc_lo, %[n1]\n"                                          \
    "s_bfe_i32 %[t0], %[t0], 0x10000\n"                                          \
    "s_xor_b32 %[v], %[v], %[t0]\n"                                              \
    "s_add_u32 %[n1], %[n1], 1\n"                                                \
    "s_lshr_b64 vcc, vcc, %[n1]\n"                                               \
    "s_sub_u32 %[nb], %[nb], %[n1]\n"                                            \
    "v_writelane_b32 %[resv], %[v], m0\n"                                        \
    "s_add_u32 m0, m0, 1\n"

// Hot code of one word of channel context C (medians M0..M2); falls through to
// the next word.  Register roles: VCC = bit window, M0 = lane of this word in
// the residual batch, h0/h1 committed early (a bail restores them: h0 was 0
// on the unary path, 1 on the holding path; h1 = ones - (u >> 1)).
#define WV2_WORD(C, M0, M1, M2)                                                  \
    "s_cmp_lt_u32 %[nb], 32\n"                                                   \
    "s_cbranch_scc1 LR" C "_%=\n"                                                \
    "LRD" C "_%=:\n"                                                             \
    "s_cmp_lg_u32 %[h0], 0\n"                                                    \
    "s_cbranch_scc1 LH" C "_%=\n"                                                \
    "s_orn2_b32 %[t0], 0x10000, vcc_lo\n"                                        \
    "s_ff1_i32_b32 %[u], %[t0]\n"                                                \
    "s_cmp_gt_u32 %[u], 15\n"                                                    \
    "s_cbranch_scc1 LX_%=\n"                                                     \
    "s_add_u32 %[c1], %[u], 1\n"                                                 \
    "s_lshr_b32 %[ones], %[u], 1\n"                                              \
    "s_add_u32 %[ones], %[ones], %[h1]\n"                                        \
    "s_and_b32 %[h1], %[u], 1\n"                                                 \
    "s_xor_b32 %[h0], %[h1], 1\n"                                                \
    "s_sub_u32 %[avail], %[nb], %[c1]\n"                                         \
    "s_cmp_lg_u32 %[ones], 0\n"                                                  \
    "s_cbranch_scc1 LG1" C "_%=\n"                                               \
    "LC0" C "_%=:\n"                                                             \
    "s_cmp_lt_i32 " M0 ", 0\n"                                                   \
    "s_cbranch_scc1 LB" C "_%=\n"                                                \
    WV2_W_BOUND(M0)                                                              \
    "s_mov_b32 %[low], 0\n"                                                      \
    WV2_W_DEC(M0, "126", "6")                                                    \
    "s_cmp_lt_u32 " M0 ", 2\n" /* zero-run mode may start: finish, then exit */  \
    "s_cbranch_scc1 LZ" C "_%=\n"                                                \
    "LT" C "_%=:\n"                                                              \
    WV2_TAIL(C, "h")

// Cold blocks of that word, placed after the loop.
#define WV2_WORD_COLD(C, M0, M1, M2, NEXT)                                       \
    /* refill from the prefetched dwords (or exit near the payload end) */        \
    "LR" C "_%=:\n"                                                              \
    "s_lshl_b32 %[t0], %[rd], 2\n"                                               \
    "s_add_u32 %[t0], %[t0], 12\n"                                               \
    "s_cmp_gt_u32 %[t0], %[E]\n"                                                 \
    "s_cbranch_scc1 LX_%=\n"                                                     \
    "s_waitcnt lgkmcnt(0)\n"                                                     \
    "s_lshl_b32 %[v], %[n0], %[nb]\n"                                            \
    "s_or_b32 vcc_lo, vcc_lo, %[v]\n"                                            \
    "s_lshr_b32 %[v], %[n0], 1\n"                                                \
    "s_sub_u32 %[u], 31, %[nb]\n"                                                \
    "s_lshr_b32 %[v], %[v], %[u]\n"                                              \
    "s_or_b32 vcc_hi, vcc_hi, %[v]\n"                                            \
    "s_add_u32 %[nb], %[nb], 32\n"                                               \
    "s_add_u32 %[rd], %[rd], 1\n"                                                \
    "s_mov_b32 %[n0], %[n1s]\n"                                                  \
    "s_sub_u32 %[t0], %[t0], 4\n"                                                \
    "s_load_dword %[n1s], %[base], %[t0]\n"                                      \
    "s_branch LRD" C "_%=\n"                                                     \
    /* holding_zero: unary count 0, h1 unchanged */                               \
    "LH" C "_%=:\n"                                                              \
    "s_mov_b32 %[c1], 0\n"                                                       \
    "s_mov_b32 %[h0], 0\n"                                                       \
    "s_mov_b32 %[ones], 0\n"                                                     \
    "s_mov_b32 %[u], 0\n"                                                        \
    "s_mov_b32 %[avail], %[nb]\n"                                                \
    "s_branch LC0" C "_%=\n"                                                     \
    "LG1" C "_%=:\n"                                                             \
    "s_cmp_eq_u32 %[ones], 1\n"                                                  \
    "s_cbranch_scc0 LG2" C "_%=\n"                                               \
    "s_cmp_lt_i32 " M1 ", 0\n"                                                   \
    "s_cbranch_scc1 LB" C "_%=\n"                                                \
    WV2_W_BOUND(M1)                                                              \
    "s_ashr_i32 %[low], " M0 ", 4\n"                                             \
    "s_add_u32 %[low], %[low], 1\n"                                              \
    WV2_W_INC(M0, "128", "7")                                                    \
    WV2_W_DEC(M1, "62", "5")                                                     \
    "s_branch LT" C "_%=\n"                                                      \
    "LG2" C "_%=:\n"                                                             \
    "s_cmp_lt_i32 " M2 ", 0\n"                                                   \
    "s_cbranch_scc1 LB" C "_%=\n"                                                \
    WV2_W_BOUND(M2)                                                              \
    "s_ashr_i32 %[low], " M0 ", 4\n"                                             \
    "s_ashr_i32 %[t0], " M1 ", 4\n"                                              \
    "s_add_u32 %[low], %[low], %[t0]\n"                                          \
    "s_add_u32 %[low], %[low], 2\n"                                              \
    WV2_W_INC(M0, "128", "7")                                                    \
    WV2_W_INC(M1, "64", "6")                                                     \
    "s_cmp_eq_u32 %[ones], 2\n"                                                  \
    "s_cbranch_scc0 LG3" C "_%=\n"                                               \
    WV2_W_DEC(M2, "30", "4")                                                     \
    "s_branch LT" C "_%=\n"                                                      \
    "LG3" C "_%=:\n"                                                             \
    "s_add_u32 %[t0], %[mc], 1\n"                                                \
    "s_sub_u32 %[v], %[ones], 2\n"                                               \
    "s_mul_i32 %[t0], %[t0], %[v]\n"                                             \
    "s_add_u32 %[low], %[low], %[t0]\n"                                          \
    WV2_W_INC(M2, "32", "5")                                                     \
    "s_branch LT" C "_%=\n"                                                      \
    /* bail before the word commits anything but h0/h1: restore them */         \
    "LB" C "_%=:\n"                                                              \
    "s_cmp_eq_u32 %[c1], 0\n"                                                    \
    "s_cbranch_scc1 LBH" C "_%=\n"                                               \
    "s_lshr_b32 %[t0], %[u], 1\n"                                                \
    "s_sub_u32 %[h1], %[ones], %[t0]\n"                                          \
    "s_mov_b32 %[h0], 0\n"                                                       \
    "s_branch LX_%=\n"                                                           \
    "LBH" C "_%=:\n"                                                             \
    "s_mov_b32 %[h0], 1\n"                                                       \
    "s_branch LX_%=\n"                                                           \
    /* this channel's median[0] dropped below 2: finish the word, then exit */  \
    "LZ" C "_%=:\n"                                                              \
    WV2_TAIL(C, "z")                                                             \
    "s_branch LE_%=\n"

// returns true when k reached kend, false when the word at k needs get_word
template <bool MONO>
__device__ __forceinline__ bool lossless_run(Entropy &w, SmemReader &rd, uint32_t &k, uint32_t kend, int32_t &resv) {
    // zero-run mode possible at the first word: general path
    if ((uint32_t)(w.med[0][0] | w.med[1][0]) < 2u) return false;
    uint32_t t0, u, ones, c1, mc, n1, low, avail, ex, v, keep;
    uint32_t nb = (uint32_t)rd.nb, rdi = rd.rd, n0 = rd.n0, n1s = rd.n1;
    int32_t m00 = w.med[0][0], m01 = w.med[0][1], m02 = w.med[0][2];
    int32_t m10 = w.med[1][0], m11 = w.med[1][1], m12 = w.med[1][2];
    int32_t h0 = w.h0, h1 = w.h1;
    const uint32_t kbase = k & ~63u;
    uint32_t lane = k - kbase;             // word index inside the batch (M0 in the loop)
    const uint32_t lend = kend - kbase;    // <= 64
    uint64_t win = rd.win;
    if (MONO) {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "LL_%=:\n"
            "s_cmp_ge_u32 m0, %[lend]\n"
            "s_cbranch_scc1 LE_%=\n"
#define C "a"
            WV2_WORD("a", "%[m00]", "%[m01]", "%[m02]")
#undef C
            "s_branch LL_%=\n"
#define C "a"
            WV2_WORD_COLD("a", "%[m00]", "%[m01]", "%[m02]", "")
#undef C
            "LX_%=:\n"
            "LE_%=:\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc), [n1] "=&s"(n1),
              [low] "=&s"(low), [avail] "=&s"(avail), [ex] "=&s"(ex), [v] "=&s"(v), [keep] "=&s"(keep),
              [win] "+s"(win), [nb] "+s"(nb), [rd] "+s"(rdi), [n0] "+s"(n0), [n1s] "+s"(n1s), [m00] "+s"(m00),
              [m01] "+s"(m01), [m02] "+s"(m02), [m10] "+s"(m10), [h0] "+s"(h0), [h1] "+s"(h1), [lane] "+s"(lane),
              [resv] "+v"(resv)
            : [lend] "s"(lend), [E] "s"(rd.E), [base] "s"(rd.base)
            : "vcc", "scc");
    } else {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "LL_%=:\n"
            "s_cmp_ge_u32 m0, %[lend]\n"
            "s_cbranch_scc1 LE_%=\n"
#define C "a"
            WV2_WORD("a", "%[m00]", "%[m01]", "%[m02]")
#undef C
#define C "b"
            WV2_WORD("b", "%[m10]", "%[m11]", "%[m12]")
#undef C
            "s_branch LL_%=\n"
#define C "a"
            WV2_WORD_COLD("a", "%[m00]", "%[m01]", "%[m02]", "")
#undef C
#define C "b"
            WV2_WORD_COLD("b", "%[m10]", "%[m11]", "%[m12]", "")
#undef C
            "LX_%=:\n"
            "LE_%=:\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc), [n1] "=&s"(n1),
              [low] "=&s"(low), [avail] "=&s"(avail), [ex] "=&s"(ex), [v] "=&s"(v), [keep] "=&s"(keep),
              [win] "+s"(win), [nb] "+s"(nb), [rd] "+s"(rdi), [n0] "+s"(n0), [n1s] "+s"(n1s), [m00] "+s"(m00),
              [m01] "+s"(m01), [m02] "+s"(m02), [m10] "+s"(m10), [m11] "+s"(m11), [m12] "+s"(m12), [h0] "+s"(h0),
              [h1] "+s"(h1), [lane] "+s"(lane), [resv] "+v"(resv)
            : [lend] "s"(lend), [E] "s"(rd.E), [base] "s"(rd.base)
            : "vcc", "scc");
    }
    rd.win = win;
    rd.nb = (int)nb;
    rd.rd = rdi;
    rd.n0 = n0;
    rd.n1 = n1s;
    w.med[0][0] = m00;
    w.med[0][1] = m01;
    w.med[0][2] = m02;
    w.med[1][0] = m10;
    w.med[1][1] = m11;
    w.med[1][2] = m12;
    w.h0 = h0;
    w.h1 = h1;
    k = kbase + lane;
    return k >= kend;
}
#undef WV2_W_BOUND
#undef WV2_W_INC
#undef WV2_W_DEC
#undef WV2_WORD
#undef WV2_WORD_COLD
#undef WV2_TAIL

// ---------------------------------------------------------------------------
// Narrow lossless run: the words of lossless_run for a batch whose entropy
// state bounds every word, so that the per-word tests of lossless_run leave
// the hot path (WordsUtils.cs:304-503 otherwise unchanged):
//   * max(med[0][0], med[1][0]) >= 66 (stereo: <= 32 updates of each
//     channel's median) or med[0][0] >= 132 (mono: <= 64) at batch start.
//     median[0] falls by m -= 2*((m+126)>>7) per update (2 while m < 130), and
//     from those starts it is still >= 2 after the batch's updates (checked
//     exhaustively): the zero-run test (:304) cannot become true inside the
//     batch -> no zero-run check per word;
//   * every median < 2^24 (stereo: <= 32 updates per channel) or < 2^22
//     (mono: <= 64) at batch start.  m += 5*((m+128)>>7) gives
//     m + 128 <= (133/128)^n (m0 + 128) (x3.4 for 32 updates, x11.7 for 64):
//     every median stays in [0, 2^25.8) (decrements never cross 0), so
//     maxcode = m >> 4 < 2^21.8, bitcount <= 22, n1 <= 21, and a word with
//     <= 7 unary ones (c1 <= 8 bits) needs c1 + n1 + 2 <= 31 bits: it fits
//     the >= 32 bits the window holds at word start, all in its low dword ->
//     no negative-median test, no window bound test.  Words with
//     8..15 unary ones (ones_count >= 4, out of line) test the bound; 16
//     (the escape, :386) leaves the run.
// The unary count and the holding_one/holding_zero pairing (:354-428) are
// branch-free (holding_zero reads no unary bits: u := 0, c1 := 0); ones == 0
// is inline, ones >= 1 out of line with its own copy of the read_code tail.
// The window refills from a 64-bit prefetch (s_load_dwordx2, one dword ahead
// of the window), and the run leaves (state intact) before a prefetch could
// read past the payload end.  Register roles as in lossless_run: VCC = bit
// window, M0 = lane of the word in the residual batch.
// ---------------------------------------------------------------------------
#define NW_DEC(M, ADD, SH1) /* m -= ((m + ADD) >> (SH1 + 1)) * 2 */ \
    "s_add_i32 %[t0], " M ", " ADD "\n"                             \
    "s_ashr_i32 %[t0], %[t0], " SH1 "\n"                            \
    "s_and_b32 %[t0], %[t0], -2\n"                                  \
    "s_sub_i32 " M ", " M ", %[t0]\n"
#define NW_INC(M, ADD, SH) /* m += ((m + ADD) >> SH) * 5 */         \
    "s_add_i32 %[t0], " M ", " ADD "\n"                             \
    "s_ashr_i32 %[t0], %[t0], " SH "\n"                             \
    "s_lshl2_add_u32 %[t0], %[t0], %[t0]\n"                         \
    "s_add_i32 " M ", " M ", %[t0]\n"
// read_code(maxcode = mc) + sign + window advance + residual into lane M0
// (WordsUtils.cs:477-503, 546-570).  z = clz(mc|1), n1 = 31 - z = bitcount-1
// (mc|1 makes maxcode 0 read no code bits), extras = 2^(n1+1) - 1 - mc.
// The scalar issue port bounds the in-flight bench, so the word
// is written for instruction count: n1 carries 0x10000 (bit offset n1, width
// 1 for s_bfe_i32: the sign as 0 / -1 in one instruction) and c1 carries
// -0x10000 (shift counts read only the low bits), so n1 + c1 is unbiased.
// nb holds (bits in the window - 32): the window advance's borrow is the next
// word's refill test (branch to NR<J>, J the next word), with no compare.
#define NW_TAIL(I, S, LOWOP, J)                                     \
    "s_or_b32 %[t0], %[mc], 1\n"                                    \
    "s_flbit_i32_b32 %[z], %[t0]\n"                                 \
    "s_lshr_b32 %[t], vcc_lo, %[c1]\n"                              \
    "s_lshr_b32 %[ex], -1, %[z]\n"                                  \
    "s_sub_u32 %[ex], %[ex], %[mc]\n"                               \
    "s_lshr_b32 %[t0], %[k7f], %[z]\n"                              \
    "s_and_b32 %[v], %[t], %[t0]\n"                                 \
    "s_sub_u32 %[n1], %[kn], %[z]\n"                                \
    "s_cmp_lt_u32 %[v], %[ex]\n"                                    \
    "s_cbranch_scc1 NS" I S "_%=\n"                                 \
    "s_lshl_b32 %[v], %[v], 1\n"                                    \
    "s_sub_u32 %[v], %[v], %[ex]\n"                                 \
    "s_bitcmp1_b32 %[t], %[n1]\n"                                   \
    "s_addc_u32 %[v], %[v], 0\n"                                    \
    "s_add_u32 %[n1], %[n1], 1\n"                                   \
    "NS" I S "_%=:\n"                                               \
    LOWOP                                                           \
    "s_bfe_i32 %[t0], %[t], %[n1]\n"                                \
    "s_xor_b32 %[v], %[v], %[t0]\n"                                 \
    "s_add_u32 %[n1], %[n1], %[c1]\n"                               \
    "s_add_u32 %[n1], %[n1], 1\n"                                   \
    "v_writelane_b32 %[resv], %[v], m0\n"                           \
    "s_add_u32 m0, m0, 1\n"                                         \
    "s_lshr_b64 vcc, vcc, %[n1]\n"                                  \
    "s_sub_u32 %[nb], %[nb], %[n1]\n" /* SCC: fewer than 32 left */ \
    "s_cbranch_scc1 NR" J "_%=\n"
// hot part of word I (channel medians MA): unary + holding flags, ones == 0
// inline; falls through to the next word.  holding_zero (:354-356: the word
// reads no unary bits, ones 0) is a virtual 0 bit shifted in front of the
// window: the unary count then finds 0 ones and c1 = u + 1 consumes the
// virtual bit (nb counts it too), with no select on h0.  The window's uncounted
// bits above nb move up one and lose bit 63; they return to their places when
// the word's shift consumes the virtual bit, and the lost bit is re-ORed by the
// next refill (at most 63 bits are counted, so bit 63 is never one of them).
#define NW_WORD(I, MA, J)                                           \
    "NA" I "_%=:\n"                                                 \
    "s_lshl_b64 vcc, vcc, %[h0]\n"                                  \
    "s_add_u32 %[nb], %[nb], %[h0]\n"                               \
    "s_orn2_b32 %[t0], %[k16], vcc_lo\n"                            \
    "s_ff1_i32_b32 %[u], %[t0]\n"                                   \
    "s_lshl1_add_u32 %[t0], %[h1], %[u]\n"                          \
    "s_and_b32 %[h1], %[u], 1\n"                                    \
    "s_add_u32 %[c1], %[u], %[kc1]\n"                               \
    "s_xor_b32 %[ex], %[h1], 1\n"                                   \
    "s_sub_u32 %[h0], %[ex], %[h0]\n"                               \
    "s_lshr_b32 %[ones], %[t0], 1\n" /* SCC = ones != 0 */          \
    "s_cbranch_scc1 NG" I "_%=\n"                                   \
    "s_lshr_b32 %[mc], " MA ", 4\n"                                 \
    NW_DEC(MA, "126", "6")                                          \
    NW_TAIL(I, "a", "", J)
// refill 32 bits from the prefetched dwords before word J, prefetch the next
// dword (or leave near the payload end), continue at DEST (the batch-end test
// in front of word J, or word J itself)
#define NW_REFILL(J, DEST)                                          \
    "NR" J "_%=:\n"                                                 \
    "s_cmp_gt_u32 %[off], %[elim]\n"                                \
    "s_cbranch_scc1 NX_%=\n"                                        \
    "s_waitcnt lgkmcnt(0)\n"                                        \
    "s_add_u32 %[nb], %[nb], 32\n" /* = bits in the window */       \
    "s_lshl_b64 %[tq], %[q], %[nb]\n"                               \
    "s_or_b64 vcc, vcc, %[tq]\n"                                    \
    "s_load_dwordx2 %[q], %[base], %[off]\n"                        \
    "s_add_u32 %[off], %[off], 4\n"                                 \
    "s_branch " DEST "_%=\n"
// cold parts of word I, placed after the loop; NEXT = label of the next word
#define NW_COLD(I, NEXT, MA, MB, MC, J)                             \
    "NG" I "_%=:\n" /* ones == 1 */                                 \
    "s_cmp_eq_u32 %[ones], 1\n"                                     \
    "s_cbranch_scc0 NH" I "_%=\n"                                   \
    "s_lshr_b32 %[low], " MA ", 4\n"                                \
    "s_add_u32 %[low], %[low], 1\n"                                 \
    "s_lshr_b32 %[mc], " MB ", 4\n"                                 \
    NW_INC(MA, "128", "7")                                          \
    NW_DEC(MB, "62", "5")                                           \
    NW_TAIL(I, "b", "s_add_u32 %[v], %[v], %[low]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "NH" I "_%=:\n" /* ones >= 2 */                                 \
    "s_lshr_b32 %[mc], " MC ", 4\n"                                 \
    "s_cmp_gt_u32 %[u], 7\n"                                        \
    "s_cbranch_scc1 NK" I "_%=\n"                                   \
    "NJ" I "_%=:\n"                                                 \
    "s_lshr_b32 %[low], " MA ", 4\n"                                \
    "s_lshr_b32 %[t0], " MB ", 4\n"                                 \
    "s_add_u32 %[low], %[low], %[t0]\n"                             \
    "s_add_u32 %[low], %[low], 2\n"                                 \
    NW_INC(MA, "128", "7")                                          \
    NW_INC(MB, "64", "6")                                           \
    "s_cmp_eq_u32 %[ones], 2\n"                                     \
    "s_cbranch_scc0 NM" I "_%=\n"                                   \
    NW_DEC(MC, "30", "4")                                           \
    NW_TAIL(I, "c", "s_add_u32 %[v], %[v], %[low]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "NM" I "_%=:\n" /* ones >= 3 */                                 \
    "s_add_u32 %[t0], %[mc], 1\n"                                   \
    "s_sub_u32 %[v], %[ones], 2\n"                                  \
    "s_mul_i32 %[t0], %[t0], %[v]\n"                                \
    "s_add_u32 %[low], %[low], %[t0]\n"                             \
    NW_INC(MC, "32", "5")                                           \
    NW_TAIL(I, "d", "s_add_u32 %[v], %[v], %[low]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "NK" I "_%=:\n" /* 8..16 unary ones: escape, or test the bound */ \
    "s_cmp_gt_u32 %[u], 15\n"                                       \
    "s_cbranch_scc1 NB" I "_%=\n"                                   \
    "s_or_b32 %[t0], %[mc], 1\n"                                    \
    "s_flbit_i32_b32 %[t0], %[t0]\n"                                \
    "s_add_u32 %[t], %[u], 1\n" /* c1 (no holding_zero here) */     \
    "s_cmp_lt_u32 %[t], %[t0]\n" /* c1 + n1 + 2 <= 32 */            \
    "s_cbranch_scc1 NJ" I "_%=\n"                                   \
    "NB" I "_%=:\n" /* leave before the word commits: restore h0/h1 */ \
    "s_lshr_b32 %[t0], %[u], 1\n"                                   \
    "s_sub_u32 %[h1], %[ones], %[t0]\n"                             \
    "s_mov_b32 %[h0], 0\n"                                          \
    "s_branch NX_%=\n"

#define NW_CHECK(L) /* batch end? */                                \
    L "_%=:\n"                                                      \
    "s_cmp_ge_u32 m0, %[lend]\n"                                    \
    "s_cbranch_scc1 NE_%=\n"

// true when the narrow run may start at this batch position (see above)
template <bool MONO>
__device__ __forceinline__ bool narrow_ok(const Entropy &w, const SmemReader &rd) {
    const int32_t mx = max(w.med[0][0], w.med[1][0]);
    const uint32_t all = (uint32_t)(w.med[0][0] | w.med[0][1] | w.med[0][2] | w.med[1][0] | w.med[1][1] | w.med[1][2]);
    return mx >= (MONO ? 132 : 66) && all < (MONO ? (1u << 22) : (1u << 24)) && rd.E >= 16u;
}

// returns true when k reached kend, false when the word at k needs get_word
template <bool MONO>
__device__ __forceinline__ bool lossless_run_narrow(Entropy &w, SmemReader &rd, uint32_t &k, uint32_t kend,
                                                    int32_t &resv) {
    uint32_t t0, t, u, ones, c1, mc, z, n1, low, ex, v, keep;
    uint64_t tq;
    uint32_t nb = (uint32_t)rd.nb;
    uint32_t off = 4u * (rd.rd + 1u);                      // byte offset of the next prefetch
    uint64_t q = (uint64_t)rd.n0 | ((uint64_t)rd.n1 << 32);  // dwords rd, rd+1
    const uint32_t elim = rd.E - 8u;
    int32_t m00 = w.med[0][0], m01 = w.med[0][1], m02 = w.med[0][2];
    int32_t m10 = w.med[1][0], m11 = w.med[1][1], m12 = w.med[1][2];
    int32_t h0 = w.h0, h1 = w.h1;
    const uint32_t kbase = k & ~63u;
    uint32_t lane = k - kbase;
    const uint32_t lend = kend - kbase;
    uint64_t win = rd.win;
    if (MONO) {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 NR0_%=\n"
            NW_CHECK("NL")
            NW_WORD("0", "%[m00]", "1")
            NW_CHECK("NC0")
            NW_WORD("1", "%[m00]", "2")
            NW_CHECK("NC1")
            NW_WORD("2", "%[m00]", "3")
            NW_CHECK("NC2")
            NW_WORD("3", "%[m00]", "0")
            "NC3_%=:\n"
            "s_branch NL_%=\n"
            NW_REFILL("0", "NL")
            NW_REFILL("1", "NC0")
            NW_REFILL("2", "NC1")
            NW_REFILL("3", "NC2")
            NW_COLD("0", "NC0", "%[m00]", "%[m01]", "%[m02]", "1")
            NW_COLD("1", "NC1", "%[m00]", "%[m01]", "%[m02]", "2")
            NW_COLD("2", "NC2", "%[m00]", "%[m01]", "%[m02]", "3")
            NW_COLD("3", "NC3", "%[m00]", "%[m01]", "%[m02]", "0")
            "NX_%=:\n"
            "NE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [t] "=&s"(t), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc),
              [z] "=&s"(z), [n1] "=&s"(n1), [low] "=&s"(low), [ex] "=&s"(ex), [v] "=&s"(v), [keep] "=&s"(keep),
              [tq] "=&s"(tq), [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off), [q] "+s"(q), [m00] "+s"(m00),
              [m01] "+s"(m01), [m02] "+s"(m02), [h0] "+s"(h0), [h1] "+s"(h1), [lane] "+s"(lane), [resv] "+v"(resv)
            : [lend] "s"(lend), [elim] "s"(elim), [base] "s"(rd.base), [k16] "s"(0x10000u), [k7f] "s"(0x7fffffffu),
              [kc1] "s"(1u - 0x10000u), [kn] "s"(0x10000u + 31u)
            : "vcc", "scc");
    } else {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 NR0_%=\n"
            "s_branch NC7_%=\n"
            "NL_%=:\n"
            NW_WORD("0", "%[m00]", "1")
            NW_WORD("1", "%[m10]", "2")
            NW_CHECK("NC1")
            NW_WORD("2", "%[m00]", "3")
            NW_WORD("3", "%[m10]", "4")
            NW_CHECK("NC3")
            NW_WORD("4", "%[m00]", "5")
            NW_WORD("5", "%[m10]", "6")
            NW_CHECK("NC5")
            NW_WORD("6", "%[m00]", "7")
            NW_WORD("7", "%[m10]", "0")
            "NC7_%=:\n"
            "s_cmp_lt_u32 m0, %[lend]\n"
            "s_cbranch_scc1 NL_%=\n"
            "s_branch NE_%=\n"
            NW_REFILL("0", "NC7")
            NW_REFILL("1", "NA1")
            NW_REFILL("2", "NC1")
            NW_REFILL("3", "NA3")
            NW_REFILL("4", "NC3")
            NW_REFILL("5", "NA5")
            NW_REFILL("6", "NC5")
            NW_REFILL("7", "NA7")
            NW_COLD("0", "NA1", "%[m00]", "%[m01]", "%[m02]", "1")
            NW_COLD("1", "NC1", "%[m10]", "%[m11]", "%[m12]", "2")
            NW_COLD("2", "NA3", "%[m00]", "%[m01]", "%[m02]", "3")
            NW_COLD("3", "NC3", "%[m10]", "%[m11]", "%[m12]", "4")
            NW_COLD("4", "NA5", "%[m00]", "%[m01]", "%[m02]", "5")
            NW_COLD("5", "NC5", "%[m10]", "%[m11]", "%[m12]", "6")
            NW_COLD("6", "NA7", "%[m00]", "%[m01]", "%[m02]", "7")
            NW_COLD("7", "NC7", "%[m10]", "%[m11]", "%[m12]", "0")
            "NX_%=:\n"
            "NE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [t] "=&s"(t), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc),
              [z] "=&s"(z), [n1] "=&s"(n1), [low] "=&s"(low), [ex] "=&s"(ex), [v] "=&s"(v), [keep] "=&s"(keep),
              [tq] "=&s"(tq), [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off), [q] "+s"(q), [m00] "+s"(m00),
              [m01] "+s"(m01), [m02] "+s"(m02), [m10] "+s"(m10), [m11] "+s"(m11), [m12] "+s"(m12), [h0] "+s"(h0),
              [h1] "+s"(h1), [lane] "+s"(lane), [resv] "+v"(resv)
            : [lend] "s"(lend), [elim] "s"(elim), [base] "s"(rd.base), [k16] "s"(0x10000u), [k7f] "s"(0x7fffffffu),
              [kc1] "s"(1u - 0x10000u), [kn] "s"(0x10000u + 31u)
            : "vcc", "scc");
    }
    rd.win = win;
    rd.nb = (int)nb;
    rd.rd = off / 4u - 1u;
    rd.n0 = (uint32_t)q;
    rd.n1 = (uint32_t)(q >> 32);
    w.med[0][0] = m00;
    w.med[0][1] = m01;
    w.med[0][2] = m02;
    w.med[1][0] = m10;
    w.med[1][1] = m11;
    w.med[1][2] = m12;
    w.h0 = h0;
    w.h1 = h1;
    k = kbase + lane;
    return k >= kend;
}

// The exp2 / log2 byte tables of the hybrid words (update_error_limit's exp2s,
// the slow-level mylog2: WordsUtils.cs:195-261, 588-646) as one VGPR each,
// dword i in lane i, read with v_readlane: the general get_word otherwise
// loads them through scalar memory on the serial chain.
struct VTab {
    int32_t v;
    __device__ __forceinline__ uint32_t byte(uint32_t i) const {
        const uint32_t dw = (uint32_t)__builtin_amdgcn_readlane(v, (int)(i >> 2));
        return (dw >> ((i & 3u) * 8u)) & 0xFFu;
    }
};
struct VTabs {
    VTab e, l;
    __device__ __forceinline__ int exp2(int i) const { return (int)e.byte((uint32_t)i); }
    __device__ __forceinline__ int log2(int i) const { return (int)l.byte((uint32_t)i); }
};

// ---------------------------------------------------------------------------
// Narrow hybrid run (HYBRID_FLAG + HYBRID_BITRATE, no HYBRID_BALANCE, zero
// bitrate deltas): the words of get_word for a batch whose entropy state
// bounds every word, as lossless_run_narrow does for lossless blocks
// (WordsUtils.cs:195-261 update_error_limit, :354-503 the word, :588-608
// mylog2).  With bitrate_delta == 0 the bitrate accumulators never move, so
// update_error_limit is a pure function of slow_level: errlim =
// exp2s(((slow + 128) >> 8) - bitrate + 0x100), 0 when that is <= 0.  It runs
// once per frame (the channel-0 word, or every mono word) before the word
// touches any state, so a word whose errlim is 0 (read_code instead of the
// bisection) can leave to get_word, which recomputes the same errlim.
// The unary part is shifted out of the window first, and the window is
// refilled right there when fewer than 32 bits remain, so the bisection and
// the sign always read from a full low dword.
// Batch bounds (hybrid_ok): no zero-run can start (median[0] as in narrow_ok); every
// median < 2^28 (mono 2^26), so for the whole batch high - low < 2^25.8 (the
// bisection at least halves it per bit: <= 26 bits + sign <= 32) and mid <
// 2^28.1; slow_level < 0x1E0000 and bitrate in [0, 0x1000]: mylog2 of such a
// mid is < 0x1E00, so slow_level's log stays <= 0x1E00 and exp2s's argument
// < 0x2000 (exponent <= 31: its shift stays inside 32 bits, errlim >= 0);
// >= 320 payload bytes left (64 words of <= 36 bits), so no refill of the
// batch reads past the payload.
// The exp2 / log2 byte tables come from VGPRs (v_readlane, VTabs).
// ---------------------------------------------------------------------------
// errlim of one channel: EL = x > 0 ? exp2s(x) : 0, x = slow_log - BR + 0x100
#define HW_EL(SLOW, BR, EL)                                         \
    "s_add_u32 %[x], " SLOW ", 128\n"                               \
    "s_ashr_i32 %[x], %[x], 8\n"                                    \
    "s_sub_i32 %[x], %[x], " BR "\n"                                \
    "s_add_i32 %[x], %[x], 0x100\n"                                 \
    "s_bfe_u32 %[b], %[x], 0x60002\n" /* dword (x & 0xff) >> 2 */   \
    "v_readlane_b32 %[t0], %[etab], %[b]\n"                         \
    "s_lshl_b32 %[b], %[x], 3\n" /* (x & 3) * 8 as a shift count */ \
    "s_lshr_b32 %[t0], %[t0], %[b]\n"                               \
    "s_and_b32 %[t0], %[t0], 0xff\n"                                \
    "s_lshl_b32 %[t0], %[t0], 22\n"                                 \
    "s_or_b32 %[t0], %[t0], %[k30]\n" /* (table | 0x100) << 22 */   \
    "s_lshr_b32 %[b], %[x], 8\n" /* exponent e <= 31 */             \
    "s_sub_u32 %[b], 31, %[b]\n"                                    \
    "s_lshr_b32 " EL ", %[t0], %[b]\n" /* e<=9: >> (9-e), else << (e-9) */ \
    "s_cmp_gt_i32 %[x], 0\n"                                        \
    "s_cselect_b32 " EL ", " EL ", 0\n"
// bisection (:477-492, high - low > errlim) on the window's low dword, sign
// (:494-497), residual into lane M0, slow_level += mylog2(mid) - ((slow +
// 128) >> 8) (:501-502), window advance; the advance's borrow is the next
// word's refill test
// The bisection runs on (low, n = high - low + 1): mid = low + (n >> 1), a 1
// bit keeps the upper ceil(n / 2) values from mid, a 0 bit the lower n >> 1
// (the reference's mid = (high + (low = mid) + 1) >> 1 / ((high = mid - 1) +
// low + 1) >> 1), and the loop runs while n > errlim + 1.  Seven scalar
// instructions and the test per bit, unrolled four bits per backward branch.
#define HW_STEP(I, S)                                               \
    "s_cmp_le_u32 %[hi], %[c1]\n"                                   \
    "s_cbranch_scc1 HD" I S "_%=\n"                                 \
    "s_lshr_b32 %[md], %[hi], 1\n"                                  \
    "s_add_u32 %[x], %[lo], %[md]\n"                                \
    "s_sub_u32 %[b], %[hi], %[md]\n"                                \
    "s_bitcmp1_b32 vcc_lo, %[kb]\n"                                 \
    "s_cselect_b32 %[lo], %[x], %[lo]\n"                            \
    "s_cselect_b32 %[hi], %[b], %[md]\n"                            \
    "s_add_u32 %[kb], %[kb], 1\n"
#define HW_TAIL(I, S, SLOW, EL, J)                                  \
    "s_mov_b32 %[kb], %[k16]\n" /* bit index, s_bfe width 1 */      \
    "s_sub_u32 %[hi], %[hi], %[lo]\n"                               \
    "s_add_u32 %[hi], %[hi], 1\n" /* n */                           \
    "s_add_u32 %[c1], " EL ", 1\n"                                  \
    "HB" I S "_%=:\n"                                               \
    HW_STEP(I, S) HW_STEP(I, S) HW_STEP(I, S) HW_STEP(I, S)         \
    "s_branch HB" I S "_%=\n"                                       \
    "HD" I S "_%=:\n"                                               \
    "s_lshr_b32 %[md], %[hi], 1\n"                                  \
    "s_add_u32 %[md], %[md], %[lo]\n" /* mid */                     \
    "s_bfe_i32 %[x], vcc_lo, %[kb]\n"                               \
    "s_xor_b32 %[b], %[md], %[x]\n"                                 \
    "v_writelane_b32 %[resv], %[b], m0\n"                           \
    "s_add_u32 m0, m0, 1\n"                                         \
    "s_lshr_b32 %[x], %[md], 9\n"                                   \
    "s_add_u32 %[x], %[md], %[x]\n" /* avalue */                    \
    "s_flbit_i32_b32 %[lo], %[x]\n"                                 \
    "s_min_u32 %[lo], %[lo], 32\n"                                  \
    "s_lshl_b32 %[x], %[x], %[lo]\n" /* leading one at bit 31 */    \
    "s_bfe_u32 %[hi], %[x], 0x60019\n" /* log2 index >> 2 */        \
    "v_readlane_b32 %[b], %[ltab], %[hi]\n"                         \
    "s_bfe_u32 %[hi], %[x], 0x20017\n"                              \
    "s_lshl_b32 %[hi], %[hi], 3\n"                                  \
    "s_lshr_b32 %[b], %[b], %[hi]\n"                                \
    "s_and_b32 %[b], %[b], 0xff\n"                                  \
    "s_sub_u32 %[lo], 32, %[lo]\n" /* dbits */                      \
    "s_lshl_b32 %[lo], %[lo], 8\n"                                  \
    "s_add_u32 %[b], %[b], %[lo]\n" /* mylog2(mid) */               \
    "s_add_u32 %[x], " SLOW ", 128\n"                               \
    "s_ashr_i32 %[x], %[x], 8\n"                                    \
    "s_sub_u32 " SLOW ", " SLOW ", %[x]\n"                          \
    "s_add_u32 " SLOW ", " SLOW ", %[b]\n"                          \
    "s_add_u32 %[c1], %[kb], %[kc1]\n" /* bisection bits + sign */  \
    "s_lshr_b64 vcc, vcc, %[c1]\n"                                  \
    "s_sub_u32 %[nb], %[nb], %[c1]\n"                               \
    "s_cbranch_scc1 HR" J "_%=\n"
// hot part of hybrid word I: errlim update (UPD), errlim == 0 or >= 8 unary
// bits -> leave, unary + holding flags (as NW_WORD), the unary bits out of the
// window (HQ: refill below 32), ones == 0 inline
#define HW_WORD(I, MA, SLOW, EL, J, UPD)                            \
    "HA" I "_%=:\n"                                                 \
    UPD                                                             \
    "s_cmp_eq_u32 " EL ", 0\n"                                      \
    "s_cbranch_scc1 HX_%=\n"                                        \
    "s_lshl_b32 %[t0], vcc_lo, %[h0]\n"                             \
    "s_orn2_b32 %[t0], %[k16], %[t0]\n"                             \
    "s_ff1_i32_b32 %[u], %[t0]\n"                                   \
    "s_cmp_gt_u32 %[u], 7\n"                                        \
    "s_cbranch_scc1 HX_%=\n"                                        \
    "s_lshl_b64 vcc, vcc, %[h0]\n"                                  \
    "s_add_u32 %[nb], %[nb], %[h0]\n"                               \
    "s_lshl1_add_u32 %[t0], %[h1], %[u]\n"                          \
    "s_and_b32 %[h1], %[u], 1\n"                                    \
    "s_xor_b32 %[b], %[h1], 1\n"                                    \
    "s_sub_u32 %[h0], %[b], %[h0]\n"                                \
    "s_add_u32 %[c1], %[u], 1\n"                                    \
    "s_lshr_b64 vcc, vcc, %[c1]\n"                                  \
    "s_sub_u32 %[nb], %[nb], %[c1]\n"                               \
    "s_cbranch_scc1 HQ" I "_%=\n"                                   \
    "HU" I "_%=:\n"                                                 \
    "s_lshr_b32 %[ones], %[t0], 1\n" /* SCC = ones != 0 */          \
    "s_cbranch_scc1 HG" I "_%=\n"                                   \
    "s_mov_b32 %[lo], 0\n"                                          \
    "s_lshr_b32 %[hi], " MA ", 4\n"                                 \
    NW_DEC(MA, "126", "6")                                          \
    HW_TAIL(I, "a", SLOW, EL, J)
// refill 32 bits (no payload-end test: hybrid_ok keeps the batch clear of it)
#define HW_REFILL(L, DEST)                                          \
    L "_%=:\n"                                                      \
    "s_waitcnt lgkmcnt(0)\n"                                        \
    "s_add_u32 %[nb], %[nb], 32\n"                                  \
    "s_lshl_b64 %[tq], %[q], %[nb]\n"                               \
    "s_or_b64 vcc, vcc, %[tq]\n"                                    \
    "s_load_dwordx2 %[q], %[base], %[off]\n"                        \
    "s_add_u32 %[off], %[off], 4\n"                                 \
    "s_branch " DEST "_%=\n"
// cold parts of hybrid word I (ones >= 1)
#define HW_COLD(I, NEXT, MA, MB, MC, SLOW, EL, J)                   \
    HW_REFILL("HQ" I, "HU" I)                                       \
    "HG" I "_%=:\n"                                                 \
    "s_lshr_b32 %[lo], " MA ", 4\n"                                 \
    "s_add_u32 %[lo], %[lo], 1\n"                                   \
    NW_INC(MA, "128", "7")                                          \
    "s_cmp_eq_u32 %[ones], 1\n"                                     \
    "s_cbranch_scc0 HH" I "_%=\n"                                   \
    "s_lshr_b32 %[hi], " MB ", 4\n"                                 \
    "s_add_u32 %[hi], %[hi], %[lo]\n"                               \
    NW_DEC(MB, "62", "5")                                           \
    HW_TAIL(I, "b", SLOW, EL, J)                                    \
    "s_branch " NEXT "_%=\n"                                        \
    "HH" I "_%=:\n" /* ones >= 2 */                                 \
    "s_lshr_b32 %[t0], " MB ", 4\n"                                 \
    "s_add_u32 %[lo], %[lo], %[t0]\n"                               \
    "s_add_u32 %[lo], %[lo], 1\n"                                   \
    NW_INC(MB, "64", "6")                                           \
    "s_lshr_b32 %[hi], " MC ", 4\n"                                 \
    "s_cmp_eq_u32 %[ones], 2\n"                                     \
    "s_cbranch_scc0 HM" I "_%=\n"                                   \
    "s_add_u32 %[hi], %[hi], %[lo]\n"                               \
    NW_DEC(MC, "30", "4")                                           \
    HW_TAIL(I, "c", SLOW, EL, J)                                    \
    "s_branch " NEXT "_%=\n"                                        \
    "HM" I "_%=:\n" /* ones >= 3: low += (ones-2) * A2 */           \
    "s_add_u32 %[t0], %[hi], 1\n"                                   \
    "s_sub_u32 %[b], %[ones], 2\n"                                  \
    "s_mul_i32 %[t0], %[t0], %[b]\n"                                \
    "s_add_u32 %[lo], %[lo], %[t0]\n"                               \
    "s_add_u32 %[hi], %[hi], %[lo]\n"                               \
    NW_INC(MC, "32", "5")                                           \
    HW_TAIL(I, "d", SLOW, EL, J)                                    \
    "s_branch " NEXT "_%=\n"
#define HW_CHECK(L)                                                 \
    L "_%=:\n"                                                      \
    "s_cmp_ge_u32 m0, %[lend]\n"                                    \
    "s_cbranch_scc1 HE_%=\n"

template <bool MONO>
__device__ __forceinline__ bool hybrid_ok(const Entropy &w, const SmemReader &rd, uint32_t flags) {
    using namespace wvf;
    if ((flags & (HYBRID_FLAG | HYBRID_BITRATE)) != (HYBRID_FLAG | HYBRID_BITRATE)) return false;
    if (!MONO && (flags & HYBRID_BALANCE)) return false;
    if ((w.dlt[0] | w.dlt[1]) != 0) return false;
    const int32_t mx = MONO ? w.med[0][0] : max(w.med[0][0], w.med[1][0]);
    const uint32_t all = (uint32_t)(w.med[0][0] | w.med[0][1] | w.med[0][2] |
                                    (MONO ? 0 : (w.med[1][0] | w.med[1][1] | w.med[1][2])));
    const uint32_t sl = MONO ? (uint32_t)w.slow[0] : max((uint32_t)w.slow[0], (uint32_t)w.slow[1]);
    const uint32_t b0 = (uint32_t)(int32_t)(w.acc[0] >> 16), b1 = MONO ? 0u : (uint32_t)(int32_t)(w.acc[1] >> 16);
    return mx >= (MONO ? 132 : 66) && all < (MONO ? (1u << 26) : (1u << 28)) && sl < 0x1E0000u && b0 <= 0x1000u &&
           b1 <= 0x1000u && rd.E >= 4u * rd.rd + 320u;
}

// returns true when k reached kend, false when the word at k needs get_word
template <bool MONO>
__device__ __forceinline__ bool hybrid_run_narrow(Entropy &w, SmemReader &rd, uint32_t &k, uint32_t kend,
                                                  int32_t &resv, const VTabs &tb) {
    uint32_t t0, u, ones, c1, lo, hi, md, kb, x, b, keep;
    uint64_t tq;
    uint32_t nb = (uint32_t)rd.nb;
    uint32_t off = 4u * (rd.rd + 1u);
    uint64_t q = (uint64_t)rd.n0 | ((uint64_t)rd.n1 << 32);
    int32_t m00 = w.med[0][0], m01 = w.med[0][1], m02 = w.med[0][2];
    int32_t m10 = w.med[1][0], m11 = w.med[1][1], m12 = w.med[1][2];
    int32_t h0 = w.h0, h1 = w.h1;
    int32_t s0 = w.slow[0], s1 = w.slow[1];
    int32_t e0 = w.errlim[0], e1 = w.errlim[1];
    const int32_t b0 = (int32_t)(w.acc[0] >> 16), b1 = (int32_t)(w.acc[1] >> 16);
    const uint32_t kbase = k & ~63u;
    uint32_t lane = k - kbase;
    const uint32_t lend = kend - kbase;
    uint64_t win = rd.win;
    if (MONO) {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 HR0_%=\n"
            HW_CHECK("HL")
            HW_WORD("0", "%[m00]", "%[s0]", "%[e0]", "1", HW_EL("%[s0]", "%[b0]", "%[e0]"))
            HW_CHECK("HC0")
            HW_WORD("1", "%[m00]", "%[s0]", "%[e0]", "0", HW_EL("%[s0]", "%[b0]", "%[e0]"))
            "HC1_%=:\n"
            "s_branch HL_%=\n"
            HW_REFILL("HR0", "HL")
            HW_REFILL("HR1", "HC0")
            HW_COLD("0", "HC0", "%[m00]", "%[m01]", "%[m02]", "%[s0]", "%[e0]", "1")
            HW_COLD("1", "HC1", "%[m00]", "%[m01]", "%[m02]", "%[s0]", "%[e0]", "0")
            "HX_%=:\n"
            "HE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [lo] "=&s"(lo), [hi] "=&s"(hi),
              [md] "=&s"(md), [kb] "=&s"(kb), [x] "=&s"(x), [b] "=&s"(b), [keep] "=&s"(keep), [tq] "=&s"(tq),
              [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off), [q] "+s"(q), [m00] "+s"(m00), [m01] "+s"(m01),
              [m02] "+s"(m02), [h0] "+s"(h0), [h1] "+s"(h1), [s0] "+s"(s0), [e0] "+s"(e0), [lane] "+s"(lane),
              [resv] "+v"(resv)
            : [lend] "s"(lend), [base] "s"(rd.base), [k16] "s"(0x10000u), [kc1] "s"(1u - 0x10000u), [b0] "s"(b0),
              [k30] "s"(1u << 30), [etab] "v"(tb.e.v), [ltab] "v"(tb.l.v)
            : "vcc", "scc");
    } else {
        asm volatile(
            "s_mov_b32 %[keep], m0\n"
            "s_mov_b32 m0, %[lane]\n"
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 HR0_%=\n"
            "s_branch HC1_%=\n"
            "HL_%=:\n"
            HW_WORD("0", "%[m00]", "%[s0]", "%[e0]", "1",
                    HW_EL("%[s0]", "%[b0]", "%[e0]") HW_EL("%[s1]", "%[b1]", "%[e1]"))
            HW_WORD("1", "%[m10]", "%[s1]", "%[e1]", "0", "")
            "HC1_%=:\n"
            "s_cmp_lt_u32 m0, %[lend]\n"
            "s_cbranch_scc1 HL_%=\n"
            "s_branch HE_%=\n"
            HW_REFILL("HR0", "HC1")
            HW_REFILL("HR1", "HA1")
            HW_COLD("0", "HA1", "%[m00]", "%[m01]", "%[m02]", "%[s0]", "%[e0]", "1")
            HW_COLD("1", "HC1", "%[m10]", "%[m11]", "%[m12]", "%[s1]", "%[e1]", "0")
            "HX_%=:\n"
            "HE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            "s_mov_b32 %[lane], m0\n"
            "s_mov_b32 m0, %[keep]\n"
            : [t0] "=&s"(t0), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [lo] "=&s"(lo), [hi] "=&s"(hi),
              [md] "=&s"(md), [kb] "=&s"(kb), [x] "=&s"(x), [b] "=&s"(b), [keep] "=&s"(keep), [tq] "=&s"(tq),
              [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off), [q] "+s"(q), [m00] "+s"(m00), [m01] "+s"(m01),
              [m02] "+s"(m02), [m10] "+s"(m10), [m11] "+s"(m11), [m12] "+s"(m12), [h0] "+s"(h0), [h1] "+s"(h1),
              [s0] "+s"(s0), [s1] "+s"(s1), [e0] "+s"(e0), [e1] "+s"(e1), [lane] "+s"(lane), [resv] "+v"(resv)
            : [lend] "s"(lend), [base] "s"(rd.base), [k16] "s"(0x10000u), [kc1] "s"(1u - 0x10000u), [b0] "s"(b0),
              [b1] "s"(b1), [k30] "s"(1u << 30), [etab] "v"(tb.e.v), [ltab] "v"(tb.l.v)
            : "vcc", "scc");
    }
    rd.win = win;
    rd.nb = (int)nb;
    rd.rd = off / 4u - 1u;
    rd.n0 = (uint32_t)q;
    rd.n1 = (uint32_t)(q >> 32);
    w.med[0][0] = m00;
    w.med[0][1] = m01;
    w.med[0][2] = m02;
    w.med[1][0] = m10;
    w.med[1][1] = m11;
    w.med[1][2] = m12;
    w.h0 = h0;
    w.h1 = h1;
    w.slow[0] = s0;
    w.slow[1] = s1;
    w.errlim[0] = e0;
    w.errlim[1] = e1;
    k = kbase + lane;
    return k >= kend;
}
#undef HW_EL
#undef HW_TAIL
#undef HW_STEP
#undef HW_WORD
#undef HW_REFILL
#undef HW_COLD
#undef HW_CHECK

// ---------------------------------------------------------------------------
// Full narrow batch (a whole 64-word batch from lane 0, narrow_ok): the
// narrow loop with the residual's value finished on the VALU.  The in-flight
// bench is bound by the SIMD's scalar issue while its VALU issue
// is half idle, and a word's sign, extra-bit value and `low` are off the serial
// chain (only the consumed bit count and the medians feed the next word): the
// scalar side keeps the extra-bit decision, the VALU builds
// ((v or 2v - ex + bit) + low) ^ sign and merges it into the residual VGPR
// with a lane mask (v_cndmask) that moves one lane per word.  With the batch
// starting at lane 0 and 64 words long, the unrolled loop's end test is the
// lane mask running out (once per 8 stereo / 4 mono words), so no M0 counter.
// Each VALU instruction reads at most one SGPR (gfx9 constant bus).
// ---------------------------------------------------------------------------
// the median updates on the VALU, the result read back into the median's SGPR
// (stereo: a channel's medians are next read two words later, by which time
// the v_readfirstlane has long completed)
#define WV2_FDEC FV_DEC
#define WV2_FINC FV_INC
#define FV_DEC(M, ADD, SH1)                                         \
    "v_mov_b32 %[vm], " M "\n"                                      \
    "v_add_u32 %[vm], " ADD ", %[vm]\n"                             \
    "v_ashrrev_i32 %[vm], " SH1 ", %[vm]\n"                         \
    "v_and_b32 %[vm], -2, %[vm]\n"                                  \
    "v_sub_u32 %[vm], " M ", %[vm]\n"                               \
    "s_nop 0\n" /* VALU VGPR write -> v_readfirstlane: 1 wait state */ \
    "v_readfirstlane_b32 " M ", %[vm]\n"
#define FV_INC(M, ADD, SH)                                          \
    "v_mov_b32 %[vm], " M "\n"                                      \
    "v_add_u32 %[vm], " ADD ", %[vm]\n"                             \
    "v_ashrrev_i32 %[vm], " SH ", %[vm]\n"                          \
    "v_lshl_add_u32 %[vm], %[vm], 2, %[vm]\n"                       \
    "v_add_u32 %[vm], " M ", %[vm]\n"                               \
    "s_nop 0\n"                                                     \
    "v_readfirstlane_b32 " M ", %[vm]\n"
#define FW_TAIL(I, S, LOWOP, J)                                     \
    "s_or_b32 %[t0], %[mc], 1\n"                                    \
    "s_flbit_i32_b32 %[z], %[t0]\n"                                 \
    "s_lshr_b32 %[t], vcc_lo, %[c1]\n"                              \
    "s_lshr_b32 %[ex], -1, %[z]\n"                                  \
    "s_sub_u32 %[ex], %[ex], %[mc]\n"                               \
    "s_lshr_b32 %[t0], %[k7f], %[z]\n"                              \
    "s_and_b32 %[v], %[t], %[t0]\n"                                 \
    "s_sub_u32 %[n1], %[kn], %[z]\n"                                \
    "v_mov_b32 %[vt], %[t]\n"                                       \
    "s_cmp_lt_u32 %[v], %[ex]\n"                                    \
    "s_cbranch_scc1 FS" I S "_%=\n"                                 \
    "v_lshlrev_b32_e64 %[r], 1, %[v]\n"                             \
    "v_subrev_u32 %[r], %[ex], %[r]\n"                              \
    "v_bfe_u32 %[rb], %[vt], %[n1], 1\n"                            \
    "v_add_u32 %[r], %[r], %[rb]\n"                                 \
    "s_add_u32 %[n1], %[n1], 1\n"                                   \
    "s_branch FT" I S "_%=\n"                                       \
    "FS" I S "_%=:\n"                                               \
    "v_mov_b32 %[r], %[v]\n"                                        \
    "FT" I S "_%=:\n"                                               \
    LOWOP                                                           \
    "v_bfe_i32 %[rb], %[vt], %[n1], 1\n"                            \
    "v_xor_b32 %[r], %[r], %[rb]\n"                                 \
    "v_cndmask_b32_e64 %[resv], %[resv], %[r], %[lm]\n"             \
    "s_lshl_b64 %[lm], %[lm], 1\n"                                  \
    "s_add_u32 %[n1], %[n1], %[c1]\n"                               \
    "s_add_u32 %[n1], %[n1], 1\n"                                   \
    "s_lshr_b64 vcc, vcc, %[n1]\n"                                  \
    "s_sub_u32 %[nb], %[nb], %[n1]\n" /* SCC: fewer than 32 left */ \
    "s_cbranch_scc1 FR" J "_%=\n"
#define FW_WORD(I, MA, J, DEC)                                           \
    "FA" I "_%=:\n"                                                 \
    "s_lshl_b64 vcc, vcc, %[h0]\n"                                  \
    "s_add_u32 %[nb], %[nb], %[h0]\n"                               \
    "s_orn2_b32 %[t0], %[k16], vcc_lo\n"                            \
    "s_ff1_i32_b32 %[u], %[t0]\n"                                   \
    "s_lshl1_add_u32 %[t0], %[h1], %[u]\n"                          \
    "s_and_b32 %[h1], %[u], 1\n"                                    \
    "s_add_u32 %[c1], %[u], %[kc1]\n"                               \
    "s_xor_b32 %[ex], %[h1], 1\n"                                   \
    "s_sub_u32 %[h0], %[ex], %[h0]\n"                               \
    "s_lshr_b32 %[ones], %[t0], 1\n" /* SCC = ones != 0 */          \
    "s_cbranch_scc1 FG" I "_%=\n"                                   \
    "s_lshr_b32 %[mc], " MA ", 4\n"                                 \
    DEC(MA, "126", "6")                                             \
    FW_TAIL(I, "a", "", J)
#define FW_REFILL(J, DEST)                                          \
    "FR" J "_%=:\n"                                                 \
    "s_cmp_gt_u32 %[off], %[elim]\n"                                \
    "s_cbranch_scc1 FX_%=\n"                                        \
    "s_waitcnt lgkmcnt(0)\n"                                        \
    "s_add_u32 %[nb], %[nb], 32\n"                                  \
    "s_lshl_b64 %[tq], %[q], %[nb]\n"                               \
    "s_or_b64 vcc, vcc, %[tq]\n"                                    \
    "s_load_dwordx2 %[q], %[base], %[off]\n"                        \
    "s_add_u32 %[off], %[off], 4\n"                                 \
    "s_branch " DEST "_%=\n"
#define FW_COLD(I, NEXT, MA, MB, MC, J, DEC, INC)                             \
    "FG" I "_%=:\n" /* ones == 1 */                                 \
    "s_cmp_eq_u32 %[ones], 1\n"                                     \
    "s_cbranch_scc0 FH" I "_%=\n"                                   \
    "s_lshr_b32 %[low], " MA ", 4\n"                                \
    "s_add_u32 %[low], %[low], 1\n"                                 \
    "s_lshr_b32 %[mc], " MB ", 4\n"                                 \
    INC(MA, "128", "7")                                          \
    DEC(MB, "62", "5")                                           \
    FW_TAIL(I, "b", "v_add_u32 %[r], %[low], %[r]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "FH" I "_%=:\n" /* ones >= 2 */                                 \
    "s_lshr_b32 %[mc], " MC ", 4\n"                                 \
    "s_cmp_gt_u32 %[u], 7\n"                                        \
    "s_cbranch_scc1 FK" I "_%=\n"                                   \
    "FJ" I "_%=:\n"                                                 \
    "s_lshr_b32 %[low], " MA ", 4\n"                                \
    "s_lshr_b32 %[t0], " MB ", 4\n"                                 \
    "s_add_u32 %[low], %[low], %[t0]\n"                             \
    "s_add_u32 %[low], %[low], 2\n"                                 \
    INC(MA, "128", "7")                                          \
    INC(MB, "64", "6")                                           \
    "s_cmp_eq_u32 %[ones], 2\n"                                     \
    "s_cbranch_scc0 FM" I "_%=\n"                                   \
    DEC(MC, "30", "4")                                           \
    FW_TAIL(I, "c", "v_add_u32 %[r], %[low], %[r]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "FM" I "_%=:\n" /* ones >= 3 */                                 \
    "s_add_u32 %[t0], %[mc], 1\n"                                   \
    "s_sub_u32 %[v], %[ones], 2\n"                                  \
    "s_mul_i32 %[t0], %[t0], %[v]\n"                                \
    "s_add_u32 %[low], %[low], %[t0]\n"                             \
    INC(MC, "32", "5")                                           \
    FW_TAIL(I, "d", "v_add_u32 %[r], %[low], %[r]\n", J)            \
    "s_branch " NEXT "_%=\n"                                        \
    "FK" I "_%=:\n" /* 8..16 unary ones: escape, or test the bound */ \
    "s_cmp_gt_u32 %[u], 15\n"                                       \
    "s_cbranch_scc1 FB" I "_%=\n"                                   \
    "s_or_b32 %[t0], %[mc], 1\n"                                    \
    "s_flbit_i32_b32 %[t0], %[t0]\n"                                \
    "s_add_u32 %[t], %[u], 1\n" /* c1 (no holding_zero here) */     \
    "s_cmp_lt_u32 %[t], %[t0]\n" /* c1 + n1 + 2 <= 32 */            \
    "s_cbranch_scc1 FJ" I "_%=\n"                                   \
    "FB" I "_%=:\n" /* leave before the word commits: restore h0/h1 */ \
    "s_lshr_b32 %[t0], %[u], 1\n"                                   \
    "s_sub_u32 %[h1], %[ones], %[t0]\n"                             \
    "s_mov_b32 %[h0], 0\n"                                          \
    "s_branch FX_%=\n"

// a whole batch (k at a batch start, 64 words to go); returns true when the
// batch is done, false when the word at k needs get_word
template <bool MONO>
__device__ __forceinline__ bool lossless_run_full(Entropy &w, SmemReader &rd, uint32_t &k, int32_t &resv) {
    uint32_t t0, t, u, ones, c1, mc, z, n1, low, ex, v;
    int32_t r, rb, vt, vm;
    uint64_t tq, lm = 1;
    uint32_t nb = (uint32_t)rd.nb;
    uint32_t off = 4u * (rd.rd + 1u);
    uint64_t q = (uint64_t)rd.n0 | ((uint64_t)rd.n1 << 32);
    const uint32_t elim = rd.E - 8u;
    int32_t m00 = w.med[0][0], m01 = w.med[0][1], m02 = w.med[0][2];
    int32_t m10 = w.med[1][0], m11 = w.med[1][1], m12 = w.med[1][2];
    int32_t h0 = w.h0, h1 = w.h1;
    uint64_t win = rd.win;
    if (MONO) {
        asm volatile(
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 FR0_%=\n"
            "FL_%=:\n"
            FW_WORD("0", "%[m00]", "1", NW_DEC)
            FW_WORD("1", "%[m00]", "2", NW_DEC)
            FW_WORD("2", "%[m00]", "3", NW_DEC)
            FW_WORD("3", "%[m00]", "0", NW_DEC)
            "FC3_%=:\n"
            "s_cmp_lg_u64 %[lm], 0\n"
            "s_cbranch_scc1 FL_%=\n"
            "s_branch FE_%=\n"
            FW_REFILL("0", "FC3")
            FW_REFILL("1", "FA1")
            FW_REFILL("2", "FA2")
            FW_REFILL("3", "FA3")
            FW_COLD("0", "FA1", "%[m00]", "%[m01]", "%[m02]", "1", NW_DEC, NW_INC)
            FW_COLD("1", "FA2", "%[m00]", "%[m01]", "%[m02]", "2", NW_DEC, NW_INC)
            FW_COLD("2", "FA3", "%[m00]", "%[m01]", "%[m02]", "3", NW_DEC, NW_INC)
            FW_COLD("3", "FC3", "%[m00]", "%[m01]", "%[m02]", "0", NW_DEC, NW_INC)
            "FX_%=:\n"
            "FE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            : [t0] "=&s"(t0), [t] "=&s"(t), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc),
              [z] "=&s"(z), [n1] "=&s"(n1), [low] "=&s"(low), [ex] "=&s"(ex), [v] "=&s"(v), [tq] "=&s"(tq),
              [r] "=&v"(r), [rb] "=&v"(rb), [vt] "=&v"(vt), [vm] "=&v"(vm), [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off),
              [q] "+s"(q), [m00] "+s"(m00), [m01] "+s"(m01), [m02] "+s"(m02), [h0] "+s"(h0), [h1] "+s"(h1),
              [lm] "+s"(lm), [resv] "+v"(resv)
            : [elim] "s"(elim), [base] "s"(rd.base), [k16] "s"(0x10000u), [k7f] "s"(0x7fffffffu),
              [kc1] "s"(1u - 0x10000u), [kn] "s"(0x10000u + 31u)
            : "vcc", "scc");
    } else {
        asm volatile(
            "s_mov_b64 vcc, %[win]\n"
            "s_sub_u32 %[nb], %[nb], 32\n"
            "s_cbranch_scc1 FR0_%=\n"
            "FL_%=:\n"
            FW_WORD("0", "%[m00]", "1", WV2_FDEC)
            FW_WORD("1", "%[m10]", "2", WV2_FDEC)
            FW_WORD("2", "%[m00]", "3", WV2_FDEC)
            FW_WORD("3", "%[m10]", "4", WV2_FDEC)
            FW_WORD("4", "%[m00]", "5", WV2_FDEC)
            FW_WORD("5", "%[m10]", "6", WV2_FDEC)
            FW_WORD("6", "%[m00]", "7", WV2_FDEC)
            FW_WORD("7", "%[m10]", "0", WV2_FDEC)
            "FC7_%=:\n"
            "s_cmp_lg_u64 %[lm], 0\n"
            "s_cbranch_scc1 FL_%=\n"
            "s_branch FE_%=\n"
            FW_REFILL("0", "FC7")
            FW_REFILL("1", "FA1")
            FW_REFILL("2", "FA2")
            FW_REFILL("3", "FA3")
            FW_REFILL("4", "FA4")
            FW_REFILL("5", "FA5")
            FW_REFILL("6", "FA6")
            FW_REFILL("7", "FA7")
            FW_COLD("0", "FA1", "%[m00]", "%[m01]", "%[m02]", "1", WV2_FDEC, WV2_FINC)
            FW_COLD("1", "FA2", "%[m10]", "%[m11]", "%[m12]", "2", WV2_FDEC, WV2_FINC)
            FW_COLD("2", "FA3", "%[m00]", "%[m01]", "%[m02]", "3", WV2_FDEC, WV2_FINC)
            FW_COLD("3", "FA4", "%[m10]", "%[m11]", "%[m12]", "4", WV2_FDEC, WV2_FINC)
            FW_COLD("4", "FA5", "%[m00]", "%[m01]", "%[m02]", "5", WV2_FDEC, WV2_FINC)
            FW_COLD("5", "FA6", "%[m10]", "%[m11]", "%[m12]", "6", WV2_FDEC, WV2_FINC)
            FW_COLD("6", "FA7", "%[m00]", "%[m01]", "%[m02]", "7", WV2_FDEC, WV2_FINC)
            FW_COLD("7", "FC7", "%[m10]", "%[m11]", "%[m12]", "0", WV2_FDEC, WV2_FINC)
            "FX_%=:\n"
            "FE_%=:\n"
            "s_add_u32 %[nb], %[nb], 32\n"
            "s_waitcnt lgkmcnt(0)\n"
            "s_mov_b64 %[win], vcc\n"
            : [t0] "=&s"(t0), [t] "=&s"(t), [u] "=&s"(u), [ones] "=&s"(ones), [c1] "=&s"(c1), [mc] "=&s"(mc),
              [z] "=&s"(z), [n1] "=&s"(n1), [low] "=&s"(low), [ex] "=&s"(ex), [v] "=&s"(v), [tq] "=&s"(tq),
              [r] "=&v"(r), [rb] "=&v"(rb), [vt] "=&v"(vt), [vm] "=&v"(vm), [win] "+s"(win), [nb] "+s"(nb), [off] "+s"(off),
              [q] "+s"(q), [m00] "+s"(m00), [m01] "+s"(m01), [m02] "+s"(m02), [m10] "+s"(m10), [m11] "+s"(m11),
              [m12] "+s"(m12), [h0] "+s"(h0), [h1] "+s"(h1), [lm] "+s"(lm), [resv] "+v"(resv)
            : [elim] "s"(elim), [base] "s"(rd.base), [k16] "s"(0x10000u), [k7f] "s"(0x7fffffffu),
              [kc1] "s"(1u - 0x10000u), [kn] "s"(0x10000u + 31u)
            : "vcc", "scc");
    }
    rd.win = win;
    rd.nb = (int)nb;
    rd.rd = off / 4u - 1u;
    rd.n0 = (uint32_t)q;
    rd.n1 = (uint32_t)(q >> 32);
    w.med[0][0] = m00;
    w.med[0][1] = m01;
    w.med[0][2] = m02;
    w.med[1][0] = m10;
    w.med[1][1] = m11;
    w.med[1][2] = m12;
    w.h0 = h0;
    w.h1 = h1;
    const uint32_t done = lm ? (uint32_t)__builtin_ctzll(lm) : 64u;  // words written (lane of the next)
    k += done;
    return done == 64u;
}
#undef FW_TAIL
#undef FW_WORD
#undef FV_DEC
#undef FV_INC
#undef WV2_FDEC
#undef WV2_FINC
#undef FW_REFILL
#undef FW_COLD
#undef NW_DEC
#undef NW_INC
#undef NW_TAIL
#undef NW_WORD
#undef NW_COLD
#undef NW_REFILL
#undef NW_CHECK

// one residual: the fast path for lossless blocks, the zero-run countdown,
// else the general get_word (wv_decode_core.h)
template <int C, bool LOSSLESS>
__device__ __forceinline__ int parse_word(Entropy &w, Reader &rd, uint32_t flags, int32_t &v, const VTabs &tb) {
    if (LOSSLESS) {
        const uint32_t m00 = (uint32_t)(w.med[0][0] | w.med[1][0]);
        const bool zr = __builtin_expect(m00 <= 1u, 0) && (w.h0 | w.h1) == 0;
        if (__builtin_expect(!zr, 1)) {
            if (__builtin_expect(rd.nb < 32, 0)) rd.refill32();
            if (__builtin_expect(fast_word<C>(w, rd, v), 1)) {
                return DEC_OK;
            }
        } else if (w.zeros_acc > 1) {  // inside a zero run (WordsUtils.cs:306-311; slow_level is dead here)
            w.zeros_acc--;
            v = 0;
            return DEC_OK;
        }
    }
    return get_word(w, rd, flags, C, C == 0, v, tb);
}

template <bool MONO, bool LOSSLESS>
__device__ __forceinline__ void parse_loop(const BlockDesc &d, Reader &rd, Entropy &w, Shared &sh, int lane) {
    const uint32_t flags = d.flags;
    VTabs tb;  // exp2 / log2 tables, dword `lane` in each lane (hybrid words)
    tb.e.v = LOSSLESS ? 0 : (int32_t)((const __attribute__((address_space(4))) uint32_t *)c_exp2_table)[lane];
    tb.l.v = LOSSLESS ? 0 : (int32_t)((const __attribute__((address_space(4))) uint32_t *)c_log2_table)[lane];
    const uint32_t total = MONO ? d.nframes : 2u * d.nframes;
    int32_t resv = 0;
    uint32_t k = 0;
    uint32_t err = 0;
    uint32_t consumed = 0;
    while (k < total) {
        const uint32_t kend = min(total, (k & ~63u) + 64u);  // next batch boundary
        while (k < kend) {
            // inside a zero run (WordsUtils.cs:304-317): the next zeros_acc - 1
            // words are 0 and change nothing but zeros_acc (slow_level is dead
            // in lossless blocks) -> a whole stretch of the batch at once
            if (LOSSLESS && __builtin_expect(w.zeros_acc > 1, 0) &&
                (uint32_t)(w.med[0][0] | w.med[1][0]) <= 1u && (w.h0 | w.h1) == 0) {
                const uint32_t n = (uint32_t)min((int64_t)(kend - k), w.zeros_acc - 1);
                const uint32_t lo = k & 63u;
                resv = ((uint32_t)lane - lo < n) ? 0 : resv;
                w.zeros_acc -= n;
                k += n;
                continue;
            }
            // the same stretch in a hybrid block: each zero word also decays its
            // channel's slow_level (WordsUtils.cs:309-313; no update_error_limit)
            if (!LOSSLESS && __builtin_expect(w.zeros_acc > 1, 0) &&
                (uint32_t)(w.med[0][0] | w.med[1][0]) <= 1u && (w.h0 | w.h1) == 0 && (w.slow[0] | w.slow[1]) >= 0) {
                const uint32_t n = (uint32_t)min((int64_t)(kend - k), w.zeros_acc - 1);
                const uint32_t lo = k & 63u;
                resv = ((uint32_t)lane - lo < n) ? 0 : resv;
                // words of channel 0 among k .. k+n-1 (stereo alternates, k even = channel 0)
                uint32_t n0 = MONO ? n : (n + 1u - (k & 1u)) / 2u, n1 = MONO ? 0u : n - n0;
                int32_t s0 = w.slow[0], s1 = w.slow[1];
                for (; n0 && s0 >= 128; n0--) s0 -= (s0 + 128) >> 8;  // below 128 it is a fixed point
                for (; n1 && s1 >= 128; n1--) s1 -= (s1 + 128) >> 8;
                w.slow[0] = s0;
                w.slow[1] = s1;
                w.zeros_acc -= n;
                k += n;
                continue;
            }
            if (LOSSLESS && (MONO || (k & 1) == 0)) {
                if (narrow_ok<MONO>(w, rd)) {
                    if ((k & 63u) == 0 && kend - k == 64u) {
                        // false: the word at k (the run stopped there) takes the general path
                        if (lossless_run_full<MONO>(w, rd, k, resv)) break;
                    } else if (lossless_run_narrow<MONO>(w, rd, k, kend, resv)) break;
                } else if (lossless_run<MONO>(w, rd, k, kend, resv)) {
                    break;
                }
            }
            if (!LOSSLESS && (MONO || (k & 1) == 0) && hybrid_ok<MONO>(w, rd, flags)) {
                if (hybrid_run_narrow<MONO>(w, rd, k, kend, resv, tb)) break;
            }

            // the word at k (and, in stereo, its pair) through the general path
            int32_t v = 0;
            int rc = DEC_OK;
            if (MONO || (k & 1) == 0) {
                rc = parse_word<0, LOSSLESS>(w, rd, flags, v, tb);
            } else {
                rc = parse_word<1, LOSSLESS>(w, rd, flags, v, tb);
            }
            if (__builtin_expect(rc != DEC_OK, 0)) {
                err = (uint32_t)rc;
                break;
            }
            resv = writelane(v, (int)(k & 63), resv);
            k++;
        }
        if (err) break;
        {
            // wait for ring space, publish the batch
            uint32_t base = (k - 1) & ~63u;
            uint32_t spins = 0;
            while (base + 64 - consumed > (uint32_t)RES_RING) {
                __builtin_amdgcn_s_sleep(2);
                consumed = uni(lds_load_acq(&sh.consumed));
                if (uni(lds_load_acq(&sh.stop))) return;  // the block was muted
                if (++spins > SPIN_LIMIT) {
                    err = DEC_TIMEOUT;
                    break;
                }
            }
            if (err) break;
            sh.res[(base % RES_RING) + lane] = resv;
            __hip_atomic_store(&sh.pos, rd.rd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            lds_publish(&sh.produced, k);
            if (uni(lds_load_acq(&sh.stop))) return;
        }
    }
    if (err) {
        // publish the complete words before the error, then the outcome
        uint32_t base = k & ~63u;
        if ((k & 63) && err != DEC_TIMEOUT) {
            uint32_t spins = 0;
            while (base + 64 - consumed > (uint32_t)RES_RING) {
                __builtin_amdgcn_s_sleep(2);
                consumed = uni(lds_load_acq(&sh.consumed));
                if (uni(lds_load_acq(&sh.stop))) return;
                if (++spins > SPIN_LIMIT) break;
            }
            // no ring space: the slots still hold unread words, so report the
            // timeout (as the main loop does) instead of overwriting them
            if (base + 64 - consumed > (uint32_t)RES_RING) err = DEC_TIMEOUT;
            else sh.res[(base % RES_RING) + lane] = resv;
        }
        lds_store_rel(&sh.produced, k);
        lds_store_rel(&sh.err, err);
    }
}

__device__ __forceinline__ void parser(const BlockDesc &d, const uint8_t *blob, Shared &sh, int lane) {
    Reader rd;
    rd.init(blob, d.bits_off, d.bits_len);
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
}

// ---------------------------------------------------------------------------
// reconstruction wave, on the vector ALU.
//
// The parser wave is scalar-issue bound and shares its SIMD's scalar issue
// slot with any other wave there, so the reconstruction runs on the VALU:
// even lanes carry channel A (left / mono), odd lanes channel B (right).
// Passes with positive terms (17, 18, 1..8) run both channels in one
// instruction; the cross-channel negative terms (-1, -2, -3) exchange values
// between lane pairs with a DPP quad permute.  All lane pairs compute the same
// values, so a wave-wide ballot of a per-frame test is that frame's verdict.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t swap_pair(int32_t x) {  // lane 2i <-> 2i+1
    return __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ int32_t iabs(int32_t x) { return x < 0 ? (int32_t)(0u - (uint32_t)x) : x; }

// weight update of positive terms (UnpackUtils.cs:747-748): w +- delta when
// both sample and input are non-zero; negative terms clamp to +-1024
// (:808-818), and |w| <= 1024 holds for them throughout (restore_weight
// range, clamped updates), so the clamp is a plain med3.
// As sign(s) * sign(x) * delta: two v_med3_i32 and two full-rate 24-bit multiplies
// (delta <= 7) instead of a compare/select per condition.
__device__ __forceinline__ int32_t vsgn(int32_t v) {  // (the compiler lowers min/max of it to compare + selects)
    int32_t r;
    asm("v_med3_i32 %0, %1, -1, 1" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ int32_t vmul24(int32_t a, int32_t b) {  // (else a v_mul_lo_u32, quarter rate)
    int32_t r;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ int32_t vupd(int32_t w, int32_t s, int32_t x, int32_t delta) {
    return wvf::add32(w, __mul24(vmul24(vsgn(s), vsgn(x)), delta));
}
__device__ __forceinline__ int32_t vupdc(int32_t w, int32_t s, int32_t x, int32_t delta) {
    return max(-1024, min(1024, vupd(w, s, x, delta)));
}

// a wave-uniform value kept in a VGPR: the reconstruction wave holds 16 passes'
// deltas, and as SGPRs they overflowed the scalar file (spilled to VGPR lanes
// and reloaded with v_readlane inside the frame loop)
__device__ __forceinline__ int32_t in_vgpr(int32_t s) {
    int32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

template <int T>
struct VPass {
    static constexpr int NH = (T >= 17) ? 2 : ((T >= 1) ? 8 : ((T < 0) ? 8 : 1));
    int32_t w;       // weight of this lane's channel
    int32_t h[NH];   // 17/18: s0,s1; 1..8 (and mono negative): ring; stereo negative: h[0]
    int32_t delta;

    __device__ __forceinline__ void init(const BlockDesc &d, int p, bool isB) {
        w = isB ? d.weight_B[p] : d.weight_A[p];
        delta = in_vgpr(d.delta[p]);
#pragma unroll
        for (int i = 0; i < NH; i++) h[i] = 0;
        if (T >= 17) {
            h[0] = isB ? d.samples_B[p][0] : d.samples_A[p][0];
            h[1] = isB ? d.samples_B[p][1] : d.samples_A[p][1];
        } else {
            // ring: slot (U - TT) & 7 is read at phase U; TT = T (1..8) or T & 7 (mono negative)
            constexpr int TT = (T >= 1) ? T : ((T & 7) == 0 ? 8 : (T & 7));
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (i < TT) h[(8 - TT + i) & 7] = isB ? d.samples_B[p][i] : d.samples_A[p][i];
        }
    }
    __device__ __forceinline__ void init_stereo_neg(const BlockDesc &d, int p, bool isB) {
        w = isB ? d.weight_B[p] : d.weight_A[p];
        delta = in_vgpr(d.delta[p]);
#pragma unroll
        for (int i = 0; i < NH; i++) h[i] = 0;
        h[0] = isB ? d.samples_B[p][0] : d.samples_A[p][0];
    }
    __device__ __forceinline__ void trunc() { w = (int16_t)w; }

    // one frame of this pass; x is the lane's channel value in and out
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &x, bool isB) {
        using namespace wvf;
        if constexpr (T == 17 || T == 18) {
            const int32_t sa = T == 17 ? sub32(mul32(2, h[0]), h[1]) : (sub32(mul32(3, h[0]), h[1]) >> 1);
            const int32_t o = add32(apply_weight(w, sa), x);
            w = vupd(w, sa, x, delta);
            h[1] = h[0];
            h[0] = o;
            x = o;
        } else if constexpr (T >= 1 && T <= 8) {
            const int32_t sa = h[(U - T) & 7];
            const int32_t o = add32(apply_weight(w, sa), x);
            w = vupd(w, sa, x, delta);
            h[U & 7] = o;
            x = o;
        } else if constexpr (T == -1) {  // A first, then B from A's result; A keeps B's output
            const int32_t s1 = add32(x, apply_weight(w, h[0]));
            const int32_t w1 = vupdc(w, h[0], x, delta);
            const int32_t y = swap_pair(s1);
            const int32_t s2 = add32(x, apply_weight(w, y));
            const int32_t w2 = vupdc(w, y, x, delta);
            const int32_t s2x = swap_pair(s2);
            x = isB ? s2 : s1;
            w = isB ? w2 : w1;
            h[0] = isB ? h[0] : s2x;
        } else if constexpr (T == -2) {  // B first, then A; B keeps A's output
            const int32_t s1 = add32(x, apply_weight(w, h[0]));
            const int32_t w1 = vupdc(w, h[0], x, delta);
            const int32_t y = swap_pair(s1);
            const int32_t s2 = add32(x, apply_weight(w, y));
            const int32_t w2 = vupdc(w, y, x, delta);
            const int32_t s2x = swap_pair(s2);
            x = isB ? s1 : s2;
            w = isB ? w1 : w2;
            h[0] = isB ? s2x : h[0];
        } else if constexpr (T == -3) {  // both, then exchange histories
            const int32_t sv = add32(x, apply_weight(w, h[0]));
            w = vupdc(w, h[0], x, delta);
            h[0] = swap_pair(sv);
            x = sv;
        }
    }
    template <int U>
    __device__ __forceinline__ void mono(int32_t &x) {
        using namespace wvf;
        if constexpr (T == 17 || T == 18) {
            const int32_t sa = T == 17 ? sub32(mul32(2, h[0]), h[1]) : (sub32(mul32(3, h[0]), h[1]) >> 1);
            const int32_t o = add32(apply_weight(w, sa), x);
            w = vupd(w, sa, x, delta);
            h[1] = h[0];
            h[0] = o;
            x = o;
        } else {
            constexpr int TT = (T >= 1 && T <= 8) ? T : ((T & 7) == 0 ? 8 : (T & 7));
            const int32_t sa = h[(U - TT) & 7];
            const int32_t o = add32(apply_weight(w, sa), x);
            w = vupd(w, sa, x, delta);
            h[U & 7] = o;
            x = o;
        }
    }
};

template <int... Ts>
struct VChain;
template <>
struct VChain<> {
    __device__ __forceinline__ void init(const BlockDesc &, int, bool, bool) {}
    __device__ __forceinline__ void trunc() {}
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &, bool) {}
    template <int U>
    __device__ __forceinline__ void mono(int32_t &) {}
};
template <int T, int... Ts>
struct VChain<T, Ts...> {
    VPass<T> p;
    VChain<Ts...> rest;
    __device__ __forceinline__ void init(const BlockDesc &d, int i, bool isB, bool mono) {
        if (T < 0 && !mono)
            p.init_stereo_neg(d, i, isB);
        else
            p.init(d, i, isB);
        rest.init(d, i + 1, isB, mono);
    }
    __device__ __forceinline__ void trunc() {
        p.trunc();
        rest.trunc();
    }
    template <int U>
    __device__ __forceinline__ void stereo(int32_t &x, bool isB) {
        p.template stereo<U>(x, isB);
        rest.template stereo<U>(x, isB);
    }
    template <int U>
    __device__ __forceinline__ void mono(int32_t &x) {
        p.template mono<U>(x);
        rest.template mono<U>(x);
    }
};

__device__ __forceinline__ bool any_lane(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }

// Output of the mute path: the whole chunk becomes fixup(0) and every later
// chunk 0 (UnpackUtils.cs:527-543, 649-664).  All lanes store.
// Values before `skip` (a seek's discard calls) are not stored.
template <int OCH>
__device__ __forceinline__ void mute_fill(uint32_t chunk_end, uint32_t nfr, int32_t z0, int32_t z1, int32_t *out,
                                          uint32_t chunk_start, uint64_t skip, int lane) {
    uint64_t a0 = (uint64_t)chunk_start * OCH, a1 = (uint64_t)chunk_end * OCH, a2 = (uint64_t)nfr * OCH;
    for (uint64_t i = a0 + lane; i < a2; i += 64) {
        int32_t v = 0;
        if (i < a1) v = (OCH == 1) ? z0 : (((i & 1) == 0) ? z0 : z1);
        if (i >= skip) out[i] = v;
    }
}

// Chunk-seam bookkeeping of the reconstruction (uniform, SALU).
struct Seams {
    uint32_t chunk_start, chunk_end, seam8, bsp, chunk, nfr;
    uint32_t pre_end, pre_chunk;  // a seek's discard calls (next_call_len in wv_desc.h)
    bool crc_stop;
};

// The lean batch's CRC in one wave sum (wv_pipe.h does the same per group):
// crc * base^n + sum base^(n-1-j) v_j over the staged values, base 9 per stereo
// frame (3 L + R) or 3 per mono value; w0/w1 are this lane's weights for o0/o1.
struct CrcBatch {
    uint32_t w0, w1, pw;
};
__device__ __forceinline__ uint32_t upow_u32(uint32_t b, uint32_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}
template <int LAYOUT>
__device__ __forceinline__ CrcBatch crc_batch_weights(int lane) {
    CrcBatch c;
    const uint32_t j = (uint32_t)lane >> 1;
    if (LAYOUT == 0) {
        c.w0 = upow_u32(9u, 31u - j) * ((lane & 1) ? 1u : 3u);
        c.w1 = 0;
        c.pw = upow_u32(9u, 32u);
    } else if (LAYOUT == 1) {
        c.w0 = upow_u32(3u, 63u - (uint32_t)lane);
        c.w1 = 0;
        c.pw = upow_u32(3u, 64u);
    } else {  // two lanes per value: the even one counts
        c.w0 = (lane & 1) ? 0u : upow_u32(3u, 63u - j);
        c.w1 = (lane & 1) ? 0u : upow_u32(3u, 31u - j);
        c.pw = upow_u32(3u, 64u);
    }
    return c;
}
__device__ __forceinline__ uint32_t wave_sum64(uint32_t x) {  // DPP row shifts + row broadcasts, lane 63
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int32_t)x, 63);
}

// One residual batch (32 stereo / 64 mono frames from t0).  LEAN: full batch,
// no chunk-seam event inside, so no per-frame seam or validity tests.  The
// steps per frame are those of decode_pcm_block in wv_decode_core.h.
template <int LAYOUT, bool LEAN, bool JOINT, bool IDENT, class CH>
__device__ __forceinline__ void recon_batch(CH &ch, const Fixup &fx, const int32_t *res, uint32_t rbase, int32_t &o0,
                                            int32_t &o1, int32_t &crc, int32_t ml, uint32_t t0, uint32_t tvalid,
                                            Seams &sm, int &mute_at, int lane, const CrcBatch &cb) {
    using namespace wvf;
    constexpr bool MONO = LAYOUT != 0;
    constexpr uint32_t BF = MONO ? 64 : 32;
    const bool isB = !MONO && (lane & 1);
    const int pair = lane >> 1;
    // LEAN: the values before fixup are staged like the outputs (in o0/o1 when the
    // fixup is the identity, else in q0/q1), so the batch's CRC is one weighted
    // wave sum at its end (CrcBatch) and the mute test of 8 frames one ballot on
    // the running max |value|; a group that mutes is replayed from the staged
    // values for the muting frame and the crc before it (the passes' state past it
    // no longer matters: the block ends muted; fixup_tail reads no stream here)
    constexpr bool BATCH_MUTE = LEAN;
    const int32_t crc_b = crc;
    int32_t q0 = 0, q1 = 0;
    for (uint32_t g = 0; g < BF / 8; g++) {
        if (!LEAN && t0 + g * 8 >= tvalid) break;
        int32_t vmx = 0;  // the group's largest |value| (iabs: INT_MIN stays negative, as the per-frame test)
        int32_t xr[8];
#pragma unroll
        for (int u = 0; u < 8; u++)
            xr[u] = MONO ? res[(rbase + g * 8 + u) % RES_RING] : res[(rbase + 2 * (g * 8 + u) + (lane & 1)) % RES_RING];
#define WV2_VFRAME(U)                                                                          \
    {                                                                                          \
        const uint32_t j = g * 8 + (U);                                                        \
        const uint32_t t = t0 + j;                                                             \
        if (LEAN || t < tvalid) {                                                              \
            int32_t x = xr[U];                                                                 \
            int32_t fl;                                                                        \
            if (MONO) {                                                                        \
                ch.template mono<U>(x);                                                        \
                if (BATCH_MUTE) {                                                              \
                    vmx = max(vmx, iabs(x));                                                   \
                } else if (LEAN) {                                                             \
                    if (__builtin_expect(any_lane(iabs(x) > ml), 0)) {                         \
                        mute_at = (int)t;                                                      \
                        break;                                                                 \
                    }                                                                          \
                    crc = add32(mul32(crc, 3), x);                                             \
                } else {                                                                       \
                    if (!sm.crc_stop && any_lane(iabs(x) > ml)) {                              \
                        const uint32_t q = sm.bsp + (t - sm.chunk_start);                      \
                        if (q != sm.chunk_end - sm.chunk_start) {                              \
                            mute_at = (int)t;                                                  \
                            break;                                                             \
                        }                                                                      \
                        sm.crc_stop = true;                                                    \
                    }                                                                          \
                    if (!sm.crc_stop) crc = add32(mul32(crc, 3), x);                           \
                }                                                                              \
                fl = x;                                                                        \
            } else {                                                                           \
                ch.template stereo<U>(x, isB);                                                 \
                const int32_t y = swap_pair(x);                                                \
                int32_t Lv = isB ? y : x, Rv = isB ? x : y;                                    \
                if (JOINT) {                                                                   \
                    Rv = sub32(Rv, Lv >> 1);                                                   \
                    Lv = add32(Lv, Rv);                                                        \
                }                                                                              \
                fl = isB ? Rv : Lv;                                                            \
                /* even lanes test L, odd lanes R: one wave-wide ballot covers both */         \
                if (BATCH_MUTE) {                                                              \
                    vmx = max(vmx, iabs(fl));                                                  \
                } else if (__builtin_expect(any_lane(iabs(fl) > ml), 0)) {                     \
                    mute_at = (int)t;                                                          \
                    break;                                                                     \
                }                                                                              \
                if (!BATCH_MUTE) crc = add32(mul32(crc, 9), add32(mul32(Lv, 3), Rv));          \
            }                                                                                  \
            if (!LEAN && (t == sm.seam8 || t == sm.chunk_end - 1)) ch.trunc();                 \
            const int32_t pre = fl;                                                            \
            if (!IDENT) fl = fixup_tail(fx, fl);                                               \
            constexpr bool STAGE_PRE = LEAN && !IDENT;                                         \
            if (LAYOUT == 1) {                                                                 \
                o0 = lane == (int)j ? fl : o0;                                                 \
                if (STAGE_PRE) q0 = lane == (int)j ? pre : q0;                                 \
            } else if (LAYOUT == 2) {                                                          \
                if (j < 32) {                                                                  \
                    o0 = pair == (int)j ? fl : o0;                                             \
                    if (STAGE_PRE) q0 = pair == (int)j ? pre : q0;                             \
                } else {                                                                       \
                    o1 = pair == (int)j - 32 ? fl : o1;                                        \
                    if (STAGE_PRE) q1 = pair == (int)j - 32 ? pre : q1;                        \
                }                                                                              \
            } else {                                                                           \
                o0 = pair == (int)j ? fl : o0;                                                 \
                if (STAGE_PRE) q0 = pair == (int)j ? pre : q0;                                 \
            }                                                                                  \
            if (!LEAN && t == sm.chunk_end - 1) {                                              \
                sm.chunk_start = t + 1;                                                        \
                const uint32_t len_ = sm.chunk_start < sm.pre_end                                       \
                                          ? min(sm.pre_chunk, sm.pre_end - sm.chunk_start) : sm.chunk;         \
                sm.chunk_end = sm.chunk_start + len_ < sm.nfr ? sm.chunk_start + len_ : sm.nfr;        \
                sm.seam8 = (!MONO && sm.chunk_end - sm.chunk_start >= 16) ? sm.chunk_start + 7 : 0xFFFFFFFFu; \
                sm.bsp = 0;                                                                    \
                sm.crc_stop = false;                                                           \
            }                                                                                  \
        }                                                                                      \
    }
        do {
            WV2_VFRAME(0) WV2_VFRAME(1) WV2_VFRAME(2) WV2_VFRAME(3) WV2_VFRAME(4) WV2_VFRAME(5) WV2_VFRAME(6)
            WV2_VFRAME(7)
        } while (0);
#undef WV2_VFRAME
        // max |v| > ml <=> some |v| > ml; the replay finds the first one
        if (BATCH_MUTE && __builtin_expect(any_lane(vmx > ml), 0)) {
            const int32_t s0 = IDENT ? o0 : q0, s1 = IDENT ? o1 : q1;
            crc = crc_b;
            for (uint32_t j = 0; j < g * 8 + 8; j++) {
                bool mute;
                if (MONO) {
                    const int32_t v = (LAYOUT == 1) ? __builtin_amdgcn_readlane(s0, (int)j)
                                                    : (j < 32 ? __builtin_amdgcn_readlane(s0, 2 * (int)j)
                                                              : __builtin_amdgcn_readlane(s1, 2 * (int)j - 64));
                    mute = j >= g * 8 && iabs(v) > ml;
                    if (!mute) crc = add32(mul32(crc, 3), v);
                } else {
                    const int32_t Lv = __builtin_amdgcn_readlane(s0, 2 * (int)j);
                    const int32_t Rv = __builtin_amdgcn_readlane(s0, 2 * (int)j + 1);
                    mute = j >= g * 8 && (iabs(Lv) > ml || iabs(Rv) > ml);
                    if (!mute) crc = add32(mul32(crc, 9), add32(mul32(Lv, 3), Rv));
                }
                if (mute) {
                    mute_at = (int)(t0 + j);
                    break;
                }
            }
            if (mute_at < 0) crc = crc_b;  // no value of the group mutes: the batch sum below
        }
        if (mute_at >= 0) break;
    }
    if (BATCH_MUTE && mute_at < 0) {
        const int32_t s0 = IDENT ? o0 : q0, s1 = IDENT ? o1 : q1;
        const uint32_t sum = wave_sum64((uint32_t)s0 * cb.w0 + (LAYOUT == 2 ? (uint32_t)s1 * cb.w1 : 0u));
        crc = (int32_t)((uint32_t)crc_b * cb.pw + sum);
    }
}

// Reconstruction-wave side of the payload prefetch: touch every 64-byte line
// from pf up to PF_AHEAD bytes past the parser's published position
// (at most 4 lines per call), so the parser's s_loads hit the CU's scalar
// cache.  Byte offsets are relative to the dword-aligned payload base and
// stay <= pf_end (the last whole dword of the payload).
__device__ __forceinline__ void scalar_prefetch(uint32_t &pf, cdw_ptr base, uint32_t pf_end, Shared &sh) {
    const uint32_t pos = uni(__hip_atomic_load(&sh.pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) * 4u;
    uint32_t tgt = pos + PF_AHEAD;
    if (tgt > pf_end) tgt = pf_end;
    if (pf > tgt) return;
    const uint32_t o0 = pf, o1 = min(pf + 64u, tgt), o2 = min(pf + 128u, tgt), o3 = min(pf + 192u, tgt);
    uint32_t d0, d1, d2, d3;
    asm volatile(
        "s_load_dword %[d0], %[b], %[o0]\n"
        "s_load_dword %[d1], %[b], %[o1]\n"
        "s_load_dword %[d2], %[b], %[o2]\n"
        "s_load_dword %[d3], %[b], %[o3]\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [d0] "=&s"(d0), [d1] "=&s"(d1), [d2] "=&s"(d2), [d3] "=&s"(d3)
        : [b] "s"(base), [o0] "s"(o0), [o1] "s"(o1), [o2] "s"(o2), [o3] "s"(o3));
    pf = (o3 + 64u) & ~63u;
}

#ifndef WV_RECON_NOP
#define WV_RECON_NOP 0
#endif
// LAYOUT 0: stereo; 1: mono (MONO_FLAG); 2: FALSE_STEREO (mono decode, 2 ints/frame)
template <int LAYOUT, int... Ts>
__device__ __forceinline__ void recon_impl(const BlockDesc &d, const uint8_t *blob, Shared &sh, int32_t *out_base, uint32_t *status_out,
                                           uint32_t *exc_out, int lane) {
    using namespace wvf;
    constexpr bool MONO = LAYOUT != 0;  // mono decode path (MONO_DATA)
    constexpr int WPF = MONO ? 1 : 2;   // residual words per frame
    constexpr int OCH = LAYOUT == 1 ? 1 : 2;
    constexpr uint32_t BF = 64 / WPF;  // frames per residual batch
    const uint32_t flags = d.flags;
    const bool joint = (flags & JOINT_STEREO) != 0;
    const int32_t ml = d.mute_limit;
    const uint32_t nfr = d.nframes;
    int32_t *out = out_base + d.out_off;
    const uint64_t skip = (uint64_t)d.pre_end * OCH;  // a seek's discarded values (not stored)

    VChain<Ts...> ch;
    ch.init(d, 0, !MONO && (lane & 1), MONO);
    Fixup fx;
    fixup_init(fx, d);
    const bool ident = fx.mode == 3 && fx.shift == 0 && !fx.lossy;  // fixup is the identity
    const CrcBatch cb = crc_batch_weights<LAYOUT>(lane);

    uint32_t status = 0;
    int32_t crc = -1;  // identical in every lane
    bool crc_garbage = false;
    Seams sm;
    sm.chunk = d.chunk;
    sm.pre_end = d.pre_end;
    sm.pre_chunk = d.pre_chunk;
    sm.nfr = nfr;
    sm.chunk_start = 0;
    sm.chunk_end = d.first_chunk < nfr ? d.first_chunk : nfr;
    sm.seam8 = (!MONO && sm.chunk_end >= 16) ? 7 : 0xFFFFFFFFu;
    sm.bsp = d.first_bsp;
    sm.crc_stop = false;
    uint32_t produced = 0;
    // scalar-cache prefetch of the parser's payload (SmemReader layout: dword-aligned base)
    const cdw_ptr pf_base = (cdw_ptr)(blob + (d.bits_off & ~(uint64_t)3));
    const uint32_t pf_end = d.bits_len + (uint32_t)(d.bits_off & 3) >= 4u ? d.bits_len + (uint32_t)(d.bits_off & 3) - 4u : 0u;
    uint32_t pf = 0;

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
            __builtin_amdgcn_s_sleep(WV2_RECON_SLEEP);
            if (++spins > RECON_SPIN_LIMIT) {
                perr = DEC_TIMEOUT;
                break;
            }
        }
        scalar_prefetch(pf, pf_base, pf_end, sh);
        // one exit for both (a second branch here costs the 16-term kernels ~110 VGPRs
        // of structurised control flow); a timeout is a handshake bug, never a
        // property of the stream, and gets its own status bit
        if (perr == DEC_EXCEPTION || perr == DEC_TIMEOUT) {
            status |= perr == DEC_EXCEPTION ? ST_EXCEPTION : ST_TIMEOUT;
            if (lane == 0) *exc_out = produced / WPF;  // block frame of the word that threw
            lds_store_rel(&sh.stop, 1);
            break;
        }
        const uint32_t tvalid = produced < need ? produced / WPF : tend;  // a bits error cuts the batch short
        int32_t o0 = 0, o1 = 0;  // staged outputs (o1: false-stereo second half)
        int mute_at = -1;
        const uint32_t rbase = t0 * WPF;
        // A full batch with no chunk-seam event inside takes the lean path.
        const uint32_t tlast = t0 + BF - 1;
        const bool seam_in = (sm.seam8 >= t0 && sm.seam8 <= tlast) ||
                             (sm.chunk_end - 1 >= t0 && sm.chunk_end - 1 <= tlast);
        const bool quirk_in =
            MONO && (sm.crc_stop || (sm.bsp > 0 && sm.chunk_end - sm.bsp >= t0 && sm.chunk_end - sm.bsp <= tlast));
#if WV_RECON_NOP  // measurement build only: the parser's throughput with a reconstruction that does nothing
        if (false) {
#else
        if (tvalid == t0 + BF && !seam_in && !quirk_in) {
#endif
            if (joint) {
                if (ident) recon_batch<LAYOUT, true, true, true>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
                else recon_batch<LAYOUT, true, true, false>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
            } else {
                if (ident) recon_batch<LAYOUT, true, false, true>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
                else recon_batch<LAYOUT, true, false, false>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
            }
        } else {
#if !WV_RECON_NOP
            if (joint) recon_batch<LAYOUT, false, true, false>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
            else recon_batch<LAYOUT, false, false, false>(ch, fx, sh.res, rbase, o0, o1, crc, ml, t0, tvalid, sm, mute_at, lane, cb);
#endif
        }
        // the batch's residuals have been read: release the ring space
        lds_publish(&sh.consumed, tend * WPF);
        // store the batch: 64 ints per instruction, one per lane
        const uint32_t nv = (mute_at >= 0 ? (uint32_t)mute_at : tvalid) - t0;
        const uint64_t base = (uint64_t)t0 * OCH;
        if ((uint32_t)lane < nv * OCH && base + lane >= skip) out[base + lane] = o0;
        if (LAYOUT == 2 && (uint32_t)lane + 64 < nv * OCH && base + 64 + lane >= skip) out[base + 64 + lane] = o1;
        const bool bits_err = tvalid < tend;
        if (mute_at >= 0 || bits_err) {
            if (bits_err && mute_at < 0) {
                status |= ST_BITS_ERROR;
                crc_garbage = true;
                if (MONO && sm.chunk_start == 0 && sm.bsp > 0) status |= ST_NONDET;
            }
            status |= ST_MUTED;
            lds_store_rel(&sh.stop, 1);
            const int32_t z0 = fixup_tail(fx, 0);
            mute_fill<OCH>(sm.chunk_end, nfr, z0, z0, out, sm.chunk_start, skip, lane);
            break;
        }
    }
    if (!(status & (ST_EXCEPTION | ST_TIMEOUT)) && nfr == d.block_samples) {
        status |= ST_CRC_CHECKED;
        if (crc_garbage || (int32_t)uni((uint32_t)crc) != d.crc) status |= ST_CRC_ERROR;
    }
    if (lane == 0) *status_out = d.fstatus | status;
}

template <int... Ts>
__device__ __forceinline__ void recon(const BlockDesc &d, const uint8_t *blob, Shared &sh, int32_t *out, uint32_t *status_out,
                                      uint32_t *exc_out, int lane) {
    const uint32_t f = d.flags;
    if (f & wvf::FALSE_STEREO)
        recon_impl<2, Ts...>(d, blob, sh, out, status_out, exc_out, lane);
    else if (f & wvf::MONO_FLAG)
        recon_impl<1, Ts...>(d, blob, sh, out, status_out, exc_out, lane);
    else
        recon_impl<0, Ts...>(d, blob, sh, out, status_out, exc_out, lane);
}

template <int... Ts>
__device__ __forceinline__ void block_2wave(const BlockDesc *descs, const uint32_t *list, const uint8_t *blob, int32_t *out,
                            uint32_t *status, uint32_t *aux) {
    __shared__ Shared sh;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    if (threadIdx.x == 0) {
        sh.produced = 0;
        sh.consumed = 0;
        sh.err = 0;
        sh.stop = 0;
        sh.pos = 0;
    }
    __syncthreads();
    if (wave == 0)
        parser(d, blob, sh, lane);
    else
        recon<Ts...>(d, blob, sh, out, &status[bi], &aux[bi], lane);
}

}  // namespace w2
}  // namespace wvg
