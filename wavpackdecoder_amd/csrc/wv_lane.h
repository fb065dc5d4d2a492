// wv_lane.h -- the lane-per-block PCM decoder for gfx950 (the throughput kernel).
//
// One lane owns one WavPack block end to end: its get_words entropy decode
// (WordsUtils.cs:272-511), its decorr passes (UnpackUtils.cs:688-1154), joint
// stereo, CRC and fixup (:549-664, :1251-1404), so one VALU instruction
// advances 64 blocks.  The two-wave kernel (wv_wave2.h) spends a whole SIMD's
// scalar port on one block's serial chain; here the same SIMD issue slot moves
// 64 chains, at the price of a longer chain per word (every word runs every
// bucket's arithmetic as selects).  With enough blocks in flight to fill the
// chip the lane kernel decodes many times more words per SIMD cycle; one small
// batch alone is latency bound either way.
//
// Payload: each lane's bitstream is staged in LDS in 16-B units (a ring of RU
// units per lane, dword k of unit slot s of lane l at ((s * 64 + l) * 4 + k)).
// A group of GF frames issues the global loads of the next units at its start
// and writes them to LDS at its end, so a load has a whole group to arrive and
// the word loop only ever reads LDS (one dword per 32 bits consumed, fetched a
// refill ahead of its use).
//
// Scope: lossless PCM blocks (stereo; or mono and false stereo, MONO) whose
// decorr term list has a compile-time instantiation, with no sticky state, wvx/wvc/exact
// float, seek discard or framing verdict.  Everything the lane does not follow
// exactly -- a zero-run length or unary escape past the window, the LIMIT_ONES
// escape, a word longer than the window, a mute, a weight that could leave
// int16 before the next check (the (short) stores at call seams are then the
// identity), medians large enough to need 64-bit bucket bounds, a ring underrun
// -- marks the block ST_REDO, and the two-wave kernel decodes it again from its
// descriptor right after (wv_pcm_2wave_redo), so results are exactly the
// two-wave kernel's, which the GPU tests hold against the oracle.
#pragma once
#include <hip/hip_runtime.h>

#include "wv_wave2.h"

namespace wvg {
namespace lane {

constexpr uint32_t ST_REDO = 1u << 15;  // internal: decode this block again on the two-wave kernel
constexpr int RU = 32;                  // ring units (16 B) per lane: 33 KiB of LDS per 64 blocks (lane_blocks: why)
constexpr int GF = 8;                   // frames per group (refill / bound-check cadence)
constexpr int NLD = 4;                  // units a lane loads per group, at most (32 bits per word sustained)
constexpr int LPAIRS = 2;               // (parser, reconstruction) wave pairs per workgroup (lane_blocks)

__device__ __forceinline__ int32_t aw(int32_t w, int32_t s) {  // apply_weight (UnpackUtils.cs:703)
    return (int32_t)(((int64_t)w * (int64_t)s + 512) >> 10);
}

// frame t (t % 8 == U): the sample-major form of decorr_stereo_pass
// (pass_stereo, wv_decode_core.h; the ring of terms 1..8 read at t & 7, written at (t + T) & 7);
// MONO: decorr_mono_pass (UnpackUtils.cs:1085-1154), channel A alone
template <int T, int U, bool MONO>
__device__ __forceinline__ void lp_frame(int32_t &wA, int32_t &wB, const int32_t dl, int32_t *hA, int32_t *hB, int32_t &L,
                                         int32_t &R) {
    using namespace wvf;
    static_assert(!MONO || T > 0, "mono lists have positive terms only");
    if constexpr (T == 17 || T == 18) {
        const int32_t sa = T == 17 ? sub32(mul32(2, hA[0]), hA[1]) : (sub32(mul32(3, hA[0]), hA[1]) >> 1);
        const int32_t oa = add32(aw(wA, sa), L);
        wA = w2::vupd(wA, sa, L, dl);
        hA[1] = hA[0];
        hA[0] = oa;
        L = oa;
        if constexpr (MONO) return;
        const int32_t sb = T == 17 ? sub32(mul32(2, hB[0]), hB[1]) : (sub32(mul32(3, hB[0]), hB[1]) >> 1);
        const int32_t ob = add32(aw(wB, sb), R);
        wB = w2::vupd(wB, sb, R, dl);
        hB[1] = hB[0];
        hB[0] = ob;
        R = ob;
    } else if constexpr (T >= 1 && T <= 8) {
        const int32_t sa = hA[U & 7];
        const int32_t oa = add32(aw(wA, sa), L);
        wA = w2::vupd(wA, sa, L, dl);
        hA[(U + T) & 7] = oa;
        L = oa;
        if constexpr (MONO) return;
        const int32_t sb = hB[U & 7];
        const int32_t ob = add32(aw(wB, sb), R);
        wB = w2::vupd(wB, sb, R, dl);
        hB[(U + T) & 7] = ob;
        R = ob;
    } else if constexpr (T == -1) {
        const int32_t sa = add32(L, aw(wA, hA[0]));
        wA = w2::vupdc(wA, hA[0], L, dl);
        L = sa;
        const int32_t o = add32(R, aw(wB, sa));
        wB = w2::vupdc(wB, sa, R, dl);
        R = o;
        hA[0] = o;
    } else if constexpr (T == -2) {
        const int32_t sb = add32(R, aw(wB, hB[0]));
        wB = w2::vupdc(wB, hB[0], R, dl);
        R = sb;
        const int32_t o = add32(L, aw(wA, sb));
        wA = w2::vupdc(wA, sb, L, dl);
        L = o;
        hB[0] = o;
    } else if constexpr (T == -3) {
        const int32_t sa = add32(L, aw(wA, hA[0]));
        wA = w2::vupdc(wA, hA[0], L, dl);
        const int32_t sb = add32(R, aw(wB, hB[0]));
        wB = w2::vupdc(wB, hB[0], R, dl);
        hB[0] = sa;
        hA[0] = sb;
        L = sa;
        R = sb;
    }
}

// one decorrelation pass, both channels in the lane (decoder order, as BlockDesc.term)
template <int T>
struct LPass {
    static constexpr int NH = (T >= 17) ? 2 : ((T >= 1) ? 8 : 1);
    int32_t wA, wB, dl;
    int32_t hA[NH], hB[NH];

    __device__ __forceinline__ void init(const BlockDesc &d, int p) {
        wA = d.weight_A[p];
        wB = d.weight_B[p];
        dl = d.delta[p];
#pragma unroll
        for (int i = 0; i < NH; i++) {
            hA[i] = d.samples_A[p][i];
            hB[i] = d.samples_B[p][i];
        }
    }
    // frame t (t % 8 == U): lp_frame
    template <int U, bool MONO>
    __device__ __forceinline__ void frame(int32_t &L, int32_t &R) {
        lp_frame<T, U, MONO>(wA, wB, dl, hA, hB, L, R);
    }
    // .wvc (HY == 2): the frame with the exact-minus-lossy differences cL / cR carried
    // along (pass_stereo_wvc, wv_decode_core.h): a pass predicting from history moves
    // both values alike; -1 / -2 predict one channel from the other's output of this
    // pass, the exact one from the exact output with the same (not yet updated) weight
    template <int U, bool MONO>
    __device__ __forceinline__ void frame_wvc(int32_t &L, int32_t &R, int32_t &cL, int32_t &cR) {
        using namespace wvf;
        if constexpr (T == -1) {
            const int32_t w0 = wB;
            frame<U, MONO>(L, R);
            cR = add32(cR, sub32(aw(w0, add32(L, cL)), aw(w0, L)));
        } else if constexpr (T == -2) {
            const int32_t w0 = wA;
            frame<U, MONO>(L, R);
            cL = add32(cL, sub32(aw(w0, add32(R, cR)), aw(w0, R)));
        } else {
            frame<U, MONO>(L, R);
        }
    }
    // could a weight leave int16 within the next group?  (the (short) stores at
    // pass-call seams, B-4, are the identity while it cannot; negative terms stay
    // within +-1024)
    __device__ __forceinline__ bool wbad() const {
        if constexpr (T < 0) return false;
        const int32_t lim = 32767 - GF * (dl < 0 ? -dl : dl);
        return max(abs(wA), abs(wB)) > lim;
    }
};

template <int... Ts>
struct LChain;
template <>
struct LChain<> {
    __device__ __forceinline__ void init(const BlockDesc &, int) {}
    template <int U, bool MONO>
    __device__ __forceinline__ void frame(int32_t &, int32_t &) {}
    template <int U, bool MONO>
    __device__ __forceinline__ void frame_wvc(int32_t &, int32_t &, int32_t &, int32_t &) {}
    __device__ __forceinline__ bool wbad() const { return false; }
};
template <int T, int... Ts>
struct LChain<T, Ts...> {
    LPass<T> p;
    LChain<Ts...> rest;
    __device__ __forceinline__ void init(const BlockDesc &d, int i) {
        p.init(d, i);
        rest.init(d, i + 1);
    }
    template <int U, bool MONO>
    __device__ __forceinline__ void frame(int32_t &L, int32_t &R) {
        p.template frame<U, MONO>(L, R);
        rest.template frame<U, MONO>(L, R);
    }
    template <int U, bool MONO>
    __device__ __forceinline__ void frame_wvc(int32_t &L, int32_t &R, int32_t &cL, int32_t &cR) {
        p.template frame_wvc<U, MONO>(L, R, cL, cR);
        rest.template frame_wvc<U, MONO>(L, R, cL, cR);
    }
    __device__ __forceinline__ bool wbad() const { return p.wbad() || rest.wbad(); }
};

// A term list read at run time (lane kernels with Ts = {LANE_RT, NS}): up to NS passes,
// the list of the pair's first block, which every lane of the pair shares (lane_block;
// a block with another list is handed back).  The passes run pass-major over a group's
// GF frames: one wave-uniform branch on a slot's term per group, each term's frames
// with the compile-time register indices of lp_frame (a slot holds every term's
// registers: LPass<1>'s two 8-entry rings).  UnpackUtils.cs:156-187 (any list of
// -3..-1, 1..8, 17, 18), :688-1154 (the passes).
constexpr int LANE_RT = 99;
template <int... Ts>
struct LaneRt {
    static constexpr int NS = 0;
};
template <int N>
struct LaneRt<LANE_RT, N> {
    static constexpr int NS = N;
};
static_assert(offsetof(BlockDesc, term) % 4 == 0, "lane_block reads a list as dwords");
template <int NS>
struct RChain {
    LPass<1> p[NS];
    uint32_t tw[4];  // the terms, four to a dword (wave-uniform)
    int32_t nt;      // (wave-uniform)
    // passes [first, first + count) of the list ptw (wave-uniform; count <= NS)
    __device__ __forceinline__ void init(const BlockDesc &d, const uint32_t *ptw, int32_t first, int32_t count) {
        // the terms from `first` on: the 16-byte list shifted down by `first` bytes (first <= 8)
        uint64_t a = (uint64_t)ptw[0] | ((uint64_t)ptw[1] << 32), b = (uint64_t)ptw[2] | ((uint64_t)ptw[3] << 32);
        const uint32_t sh = 8u * (uint32_t)first;
        if (sh >= 64u) {
            a = b >> (sh - 64u);
            b = 0;
        } else if (sh) {
            a = (a >> sh) | (b << (64u - sh));
            b >>= sh;
        }
        tw[0] = (uint32_t)a;
        tw[1] = (uint32_t)(a >> 32);
        tw[2] = (uint32_t)b;
        tw[3] = (uint32_t)(b >> 32);
        nt = count;
#pragma unroll
        for (int i = 0; i < NS; i++) {
            p[i].init(d, min(first + i, MAXP - 1));
            if (i >= nt) p[i].wA = p[i].wB = p[i].dl = 0;  // (wbad: a slot past the list)
        }
    }
    __device__ __forceinline__ int term(int i) const { return (int32_t)(int8_t)(tw[i >> 2] >> (8 * (i & 3))); }
    template <int T, bool MONO>
    __device__ __forceinline__ static void run(LPass<1> &q, int32_t (&L)[GF], int32_t (&R)[GF]) {
        if constexpr (MONO && T < 0) {
            return;  // (lane_ok: a mono list has positive terms only)
        } else {
            lp_frame<T, 0, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[0], R[0]);
            lp_frame<T, 1, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[1], R[1]);
            lp_frame<T, 2, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[2], R[2]);
            lp_frame<T, 3, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[3], R[3]);
            lp_frame<T, 4, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[4], R[4]);
            lp_frame<T, 5, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[5], R[5]);
            lp_frame<T, 6, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[6], R[6]);
            lp_frame<T, 7, MONO>(q.wA, q.wB, q.dl, q.hA, q.hB, L[7], R[7]);
        }
    }
    // the group's GF frames through passes I.. (frame t of the group at index t % GF;
    // template recursion: every slot's registers at compile-time indices)
    template <int I, bool MONO>
    __device__ __forceinline__ void group_from(int32_t (&L)[GF], int32_t (&R)[GF]) {
        if constexpr (I < NS) {
            if (I >= nt) return;
            switch (term(I)) {
            case 1: run<1, MONO>(p[I], L, R); break;
            case 2: run<2, MONO>(p[I], L, R); break;
            case 3: run<3, MONO>(p[I], L, R); break;
            case 4: run<4, MONO>(p[I], L, R); break;
            case 5: run<5, MONO>(p[I], L, R); break;
            case 6: run<6, MONO>(p[I], L, R); break;
            case 7: run<7, MONO>(p[I], L, R); break;
            case 8: run<8, MONO>(p[I], L, R); break;
            case 17: run<17, MONO>(p[I], L, R); break;
            case 18: run<18, MONO>(p[I], L, R); break;
            case -1: run<-1, MONO>(p[I], L, R); break;
            case -2: run<-2, MONO>(p[I], L, R); break;
            default: run<-3, MONO>(p[I], L, R); break;
            }
            group_from<I + 1, MONO>(L, R);
        }
    }
    template <bool MONO>
    __device__ __forceinline__ void group(int32_t (&L)[GF], int32_t (&R)[GF]) {
        group_from<0, MONO>(L, R);
    }
    // (negative terms' weights stay within +-1024: the test holds for them too)
    __device__ __forceinline__ bool wbad() const {
        bool b = false;
#pragma unroll
        for (int i = 0; i < NS; i++) b |= p[i].wbad();
        return b;
    }
};

template <int... Ts>
struct ChainOf {
    using type = LChain<Ts...>;
};
template <int N>
struct ChainOf<LANE_RT, N> {
    using type = RChain<N>;
};

// The 64 lanes' rings are interleaved by dword: dword k of a lane's stream (a count
// of dwords from its 16-B aligned base) sits in ring slot (~k) % (4 RU), and slot p of
// lane l at byte (p * 64 + l) * 4 of its pair's ring (RING_BYTES each, one array for
// the workgroup) -- every lane's read of its next dword, whatever its position, hits
// bank l (no conflicts).  The read position is the byte offset itself (LState.ra:
// pair ring, slot, lane); the advance to the next dword is one v_lshl_add and one
// v_bfi that keeps the slot bits (RSLOT) inside the ring.  (The slots run downwards
// so that a unit's four dwords sit in four consecutive slots.)
constexpr uint32_t RING_BYTES = RU * 16u * 64u;
constexpr uint32_t RSLOT = (RU * 4u - 1u) << 8;
static_assert((RING_BYTES & (RING_BYTES - 1u)) == 0u && RSLOT == RING_BYTES - 256u, "ring layout");
__device__ __forceinline__ uint32_t rslot(uint32_t k) { return ((~k) << 8) & RSLOT; }
// ra after moving `adv` (0 or 1) dwords on, given as 0 / ~0 (a lane mask value)
__device__ __forceinline__ uint32_t ring_step(uint32_t ra, uint32_t adv_mask) {
    const uint32_t n = ra + (adv_mask << 8);
    return (n & RSLOT) | (ra & ~RSLOT);
}
// unit u (dwords 4u..4u+3) of the lane whose column is `col` (pair ring + lane * 4)
__device__ __forceinline__ uint32_t unit_addr(uint32_t col, uint32_t u) {
    return rslot(4u * u + 3u) | col;  // dword 4u + 3: the lowest of the four slots
}
__device__ __forceinline__ void put_unit_at(uint8_t *ring, uint32_t a, uint4 v) {
    *(uint32_t *)(ring + a + 768u) = v.x;
    *(uint32_t *)(ring + a + 512u) = v.y;
    *(uint32_t *)(ring + a + 256u) = v.z;
    *(uint32_t *)(ring + a) = v.w;
}
__device__ __forceinline__ void put_unit(uint8_t *ring, uint32_t col, uint32_t u, uint4 v) {
    const uint32_t a = unit_addr(col, u);
    *(uint32_t *)(ring + a + 768u) = v.x;
    *(uint32_t *)(ring + a + 512u) = v.y;
    *(uint32_t *)(ring + a + 256u) = v.z;
    *(uint32_t *)(ring + a) = v.w;
}

// bytes at or past the stream end read as 0xFF (BitsUtils.cs:125-139): unit u
// relative to a stream ending at byte e (branch-free: the real bytes of v, 0..4,
// keep their value)
__device__ __forceinline__ uint32_t ff_tail(uint32_t v, uint32_t pos, uint32_t e) {
    const uint32_t keep = min(e > pos ? e - pos : 0u, 4u);
    return v | (uint32_t)(0xFFFFFFFFFFFFFFFFull << (keep * 8u));
}
__device__ __forceinline__ uint4 ff_unit(uint4 v, uint32_t u, uint32_t e) {
    const uint32_t b = u * 16u;
    v.x = ff_tail(v.x, b, e);
    v.y = ff_tail(v.y, b + 4, e);
    v.z = ff_tail(v.z, b + 8, e);
    v.w = ff_tail(v.w, b + 12, e);
    return v;
}

// .wvc correction stream window (HY == 2; cwin_init / cwin_merge / cwin_corr below)
struct CWin {
    const uint4 *src;   // the stream's 16-B aligned base
    uint8_t *lds;       // the correction rings (WRING_OFF)
    uint32_t col;       // this lane's column of its pair's ring (byte offset from lds)
    uint64_t win;       // LSB = next bit
    int32_t nb;         // valid bits (>= 33 at every word start)
    uint32_t rd;        // index of the dword merged next (its value read ahead in nxt)
    uint32_t nxt;
    uint32_t lu;        // units (16 B) staged in the ring so far; dwords below 4 lu are readable
    uint32_t ulast;     // the stream's last unit (units past it re-read it)
    uint32_t lim;       // 4 lu at the group's start: a merge of dword rd >= lim is an underrun
    uint32_t ovf;       // an underrun happened (the block goes back)
    uint32_t used;      // bits consumed (checked against end at the block's end)
    uint32_t end;       // the stream's bits (from its first bit)
};

struct LState {
    uint64_t win;  // bit window, LSB = next bit; bits at or above nb are zero
    int32_t nb;    // valid bits in win (>= 33 at every word start)
    uint32_t ra;   // ring byte offset of the stream dword merged next (ring_step)
    uint32_t nxt;  // that dword, read ahead
    uint32_t rp;   // that dword's index k, as of the group's start (rpos: now)
    uint32_t ra0;  // ra at the group's start
    uint32_t keep;      // holding_zero as a lane mask: 0 when the next word holds a zero, else ~0
    uint32_t h1;        // holding_one as 0/1 (VGPRs: the fast words never turn a lane value into an
                        // SGPR mask and back, ~20 cycles each way)
    uint32_t zacc;
    int32_t m[2][3];
    uint32_t pmax;   // 17: a bits error or a count too long for the lane (else smaller)
    uint32_t rare;   // fast words: nonzero when a word needed the checked path (escape, run length)
    uint32_t rmax;   // no-run words: the largest raw unary count (16: an escape -> the checked path)
    uint32_t r0;     // plain no-run words (WV_LANE_SPEC): the next word's raw unary count
    int32_t slack;   // least window bits left after a word (< 0: a word past the window)
    uint32_t bad;
    uint32_t bad0;   // (diagnostics) the reasons of the first group that set any: status bits 24-31
    uint32_t bal;    // hybrid stereo with HYBRID_BALANCE: ~0 (lhy_errlim), else 0
    uint32_t nobr;   // hybrid without HYBRID_BITRATE: ~0 (the error limit is exp2s(bitrate) alone), else 0
    // hybrid words (HYBRID_FLAG | HYBRID_BITRATE): slow_level, bitrate_acc/delta, error limit per channel
    int32_t slow[2];
    int64_t acc[2], dlt[2];
    int32_t el[2];
};

// Selects on lane masks (uint64_t in SGPRs, from ballots).  WV_LANE_ASM=1 forces
// each one into a hand-written v_cndmask; the default lets the compiler emit the
// same instructions and schedule them (the hazard recognizer puts an s_nop after
// nearly every inline asm statement that feeds a VALU).
#ifndef WV_LANE_ASM
#define WV_LANE_ASM 0
#endif
__device__ __forceinline__ uint64_t lmask(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ bool lbit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
#if WV_LANE_ASM
__device__ __forceinline__ uint32_t vselm(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t addc(uint32_t a, uint64_t carry) {  // a + (this lane's bit of carry)
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(a), "s"(carry));
    return r;
}
template <int A, int B>
__device__ __forceinline__ int32_t csel(uint64_t m) {  // m ? A : B, inline constants
    int32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "i"(B), "i"(A), "s"(m));
    return r;
}
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) {  // a * b + c, 24-bit signed operands
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
#else
__device__ __forceinline__ uint32_t vselm(uint64_t m, uint32_t a, uint32_t b) { return lbit(m) ? a : b; }
__device__ __forceinline__ uint32_t addc(uint32_t a, uint64_t carry) { return a + (lbit(carry) ? 1u : 0u); }
template <int A, int B>
__device__ __forceinline__ int32_t csel(uint64_t m) { return lbit(m) ? A : B; }
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) { return __mul24(a, b) + c; }
#endif
__device__ __forceinline__ int32_t vselmi(uint64_t m, int32_t a, int32_t b) {
    return (int32_t)vselm(m, (uint32_t)a, (uint32_t)b);
}
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) { return vselm(lmask(c), a, b); }
// v_mul_u32_u24 whatever the compiler knows of the operands' range (__umul24 masks them
// first and may become v_mul_lo_u32, a quarter-rate instruction)
extern "C" __device__ uint32_t wv_lane_mul_u24(uint32_t a, uint32_t b) __asm("llvm.amdgcn.mul.u24");
__device__ __forceinline__ uint32_t mul_u24(uint32_t a, uint32_t b) { return wv_lane_mul_u24(a, b); }
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) { return a + b + c; }

// window refill: keep >= 32 bits by merging the dword read ahead (then read the next)
__device__ __forceinline__ void lrefill(LState &s, const uint8_t *ring, uint32_t rbase) {
    const bool need = s.nb <= 32;
    s.win |= (uint64_t)vsel(need, s.nxt, 0u) << ((uint32_t)s.nb & 63u);
    s.nb += need ? 32 : 0;
    s.ra = ring_step(s.ra, need ? ~0u : 0u);
    s.nxt = *(const uint32_t *)(ring + s.ra);
}
__device__ __forceinline__ void lskip(LState &s, uint32_t n) {  // consume n <= 63 bits
    s.win >>= n;
    s.nb -= (int32_t)n;
    s.slack = min(s.slack, s.nb);
}
// an Elias-gamma count (the zero-run length, WordsUtils.cs:321-335, and the
// LIMIT_ONES escape, :391-407): cb ones, a zero, cb - 1 mantissa bits below an
// implied top bit; counts of 2^30 and more (33 ones: the reference's bits error)
// go to the two-wave kernel
__device__ __forceinline__ uint32_t lgamma(LState &s, const uint8_t *ring, uint32_t rbase) {
    const uint32_t cb = (uint32_t)__builtin_ctz(~(uint32_t)s.win | 0x80000000u);  // <= 31
    if (cb >= 31u) s.pmax = 17u;
    lskip(s, cb + 1u);
    lrefill(s, ring, rbase);
    if (cb < 2u) return cb;
    const uint32_t v = ((uint32_t)s.win & ((1u << (cb - 1u)) - 1u)) | (1u << (cb - 1u));
    lskip(s, cb - 1u);
    lrefill(s, ring, rbase);
    return v;
}

// ---- hybrid words (HYBRID_FLAG with HYBRID_BITRATE, stereo) ----
// The exp2 / log2 byte tables (WordsUtils.cs) in LDS after the payload rings.
constexpr uint32_t TAB_EXP2 = LPAIRS * RING_BYTES, TAB_LOG2 = TAB_EXP2 + 256u;
// a unit a lane does not take this group (no room in its ring) is written here instead
// (4 slots of 64 lanes: every lane's put_unit_at stays branch-free)
constexpr uint32_t RING_DUMMY = TAB_LOG2 + 256u, LDS_AFTER_RINGS = 512u + 1024u;
// exp2s(L) for L > 0 (WordsUtils.cs:633-646): value (9 bits) scaled by 2^(e - 9) as
// one shift pair, exact for e <= 22 (else the lane hands its block back); 0 for L <= 0.
// L = slow_log - bitrate + 0x100: unsigned, [0x1700, 2^31 + 0x100) holds every e > 22 and
// the sums whose + 0x100 wrapped past INT_MAX (the reference's exp2s of a negative):
// one compare hands both back
__device__ __forceinline__ int32_t lexp2s_pos(int32_t L, const uint8_t *ring, uint32_t &bad) {
    const uint32_t e = (uint32_t)L >> 8;
    const uint32_t v = (uint32_t)ring[TAB_EXP2 + ((uint32_t)L & 0xFFu)] | 0x100u;
    bad |= ((uint32_t)L - 0x1700u < 0x80000100u - 0x1700u) ? 2u : 0u;
    return L > 0 ? (int32_t)((v << (e & 31u)) >> 9) : 0;
}
// update_error_limit (WordsUtils.cs:195-261): before the first word of a frame, in lanes
// where that word is not a zero-run zero.  HYBRID_BITRATE: exp2s(slow_log - bitrate + 0x100);
// stereo with HYBRID_BALANCE (:222-241) moves bitrate between the channels by their slow
// levels (a wave-uniform branch: some lane balances).  Without HYBRID_BITRATE (s.nobr):
// exp2s(bitrate) (:209, :256-258) -- a negative bitrate (the reference's exp2s of a negative:
// a negative error limit) hands the block back.  Mono and false stereo (:199-209) use
// channel 0 alone -- the lane computes channel 1 too, unused (its descriptor values are zero)
__device__ __forceinline__ void lhy_errlim(LState &s, const uint8_t *ring, bool apply) {
    using namespace wvf;
    int64_t acc[2];
    int32_t br[2], sl[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        acc[c] = s.acc[c] + s.dlt[c];
        br[c] = (int32_t)(acc[c] >> 16);
        sl[c] = add32(s.slow[c], SLO) >> SLS;
    }
    if (lmask(s.bal != 0u) != 0ull) {
        const int32_t bl = add32(add32(sub32(sl[1], sl[0]), br[1]), 1) >> 1;
        const bool up = bl > br[0], dn = sub32(0, bl) > br[0];
        const int32_t n1 = up ? mul32(br[0], 2) : (dn ? 0 : add32(br[0], bl));
        const int32_t n0 = up ? 0 : (dn ? mul32(br[0], 2) : sub32(br[0], bl));
        br[1] = s.bal ? n1 : br[1];
        br[0] = s.bal ? n0 : br[0];
    }
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int32_t L = s.nobr ? br[c] : add32(sub32(sl[c], br[c]), 0x100);
        s.bad |= s.nobr & ((uint32_t)br[c] >> 30) & 2u;  // (bit 31: a negative bitrate)
        const int32_t el = lexp2s_pos(L, ring, s.bad);
        s.acc[c] = apply ? acc[c] : s.acc[c];
        s.el[c] = apply ? el : s.el[c];
    }
}
// a hybrid word's magnitude from the 32 bits x after its unary part: read_code(high -
// low) + low when the error limit is 0, else the bisection (:486-492) -- one bit per
// step while high - low > error_limit.  The bisection runs on (lo, n = high - low + 1):
// mid = lo + (n >> 1), a 1 bit keeps the upper n - (n >> 1) values, a 0 bit the lower
// n >> 1 -- taken in closed form below, four steps per test of the wave's exit condition
// (a lane with fewer steps adds zeros).  The reference's 64-bit bounds: the lane hands
// back a word whose high reaches 2^31.
template <int HY>
__device__ __forceinline__ void lhy_code(uint32_t x, uint32_t low, uint32_t mc, int32_t el, uint32_t &mid,
                                         uint32_t &used, uint32_t &bad, uint32_t &lo_f, uint32_t &n_f) {
    const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
    const uint32_t ex = (0xFFFFFFFFu >> z) - mc;
    const uint32_t nbt = z ^ 31u;
    const uint32_t v = __builtin_amdgcn_ubfe(x, 0, nbt);
    const bool big = v >= ex;
    const uint32_t t = v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex;
    const uint32_t mid_rc = add3(low, v, big ? t : 0u);
    const uint32_t used_rc = nbt + (big ? 1u : 0u);
    const uint32_t E = (uint32_t)el + 1u;
    uint32_t lo, n, k;
    if constexpr (HY == 2) {
        // (.wvc lanes: the step loop, one bit per step -- measured faster there: 30.9 vs 31.8 ms
        // for C4 + .wvc, where the closed form below takes C4 alone 25.6 -> 24.9 ms)
        lo = low;
        n = mc + 1u;
        k = 0u;
        uint32_t am = (el != 0 && n > E) ? ~0u : 0u;
        for (uint32_t j = 0; lmask(am != 0u) != 0ull; j += 4u) {
#pragma unroll
            for (uint32_t u = 0; u < 4u; u++) {
                const uint32_t h = n >> 1;
                const uint32_t bm = (uint32_t)__builtin_amdgcn_sbfe((int32_t)x, j + u, 1);
                lo += bm & am & h;
                const uint32_t nn = h + (bm & n & 1u);
                n = (am & nn) | (~am & n);
                k -= am;
                am = n > E ? am : 0u;
            }
        }
        bad |= k > 31u ? 2u : 0u;
        k = min(k, 31u);
    } else {
        // The bisection in closed form (no step waits for the one before it): with n_i the
        // interval after i steps and B_i the first i step bits (x's low bits), n_i = (n + B_i) >> i
        // and the low end moves by (n + B_i) >> (i + 1) at every 1 bit; the steps run while
        // n_i > error_limit + 1 = E, i.e. k of them, k the first i with n_i <= E: i1 (the first i
        // with (n >> i) <= E, from the bit lengths) or i1 + 1.  (k <= 31: n < 2^31.)
        const uint32_t n0 = mc + 1u;
        const bool act = el != 0 && n0 > E;
        const uint32_t d = act ? (uint32_t)(__builtin_clz(E) - __builtin_clz(n0 | 1u)) : 0u;
        const uint32_t i1 = d + ((n0 >> d) > E ? 1u : 0u);
        const uint32_t t1 = (n0 + __builtin_amdgcn_ubfe(x, 0, i1)) >> i1;
        k = act ? i1 + (t1 > E ? 1u : 0u) : 0u;
        const uint32_t xk = __builtin_amdgcn_ubfe(x, 0, k);  // the step bits
        uint32_t acc = 0u;
        for (uint32_t j = 0; lmask(j < k) != 0ull; j += 4u) {  // (uniform: the wave's most steps)
#pragma unroll
            for (uint32_t u = 0; u < 4u; u++) {
                const uint32_t i = min(j + u, 31u);  // (bit 31 of xk is 0: k <= 31)
                const uint32_t term = (n0 + (xk & ((1u << i) - 1u))) >> min(i + 1u, 31u);
                acc += term & (uint32_t)__builtin_amdgcn_sbfe((int32_t)xk, i, 1);
            }
        }
        lo = low + acc;
        n = (n0 + xk) >> k;
    }
    bad |= ((low | (low + mc)) >= 0x80000000u) ? 2u : 0u;
    mid = el == 0 ? mid_rc : lo + (n >> 1);
    used = el == 0 ? used_rc : k;
    lo_f = lo;  // the final interval [lo, lo + n - 1] (the .wvc code's range)
    n_f = n;
}

// ---- .wvc correction stream (HY == 2; beyond the reference: WavPack 4's get_word) ----
// A hybrid word the error limit left inexact (el != 0) reads its exact magnitude as
// read_code(wvcbits, high - low) + low from the block's ID_WVC_BITSTREAM.  The parser
// hands the reconstruction wave each word's final interval (LW.clo / cn); that wave
// reads the correction, exact minus lossy, and carries it through the passes
// (LPass::frame_wvc), off the parser's chain.  Each lane reads its correction stream through a
// 64-bit register window refilled from an LDS ring (below); a lane whose reads pass the
// stream's end, or the units staged so far, hands its block back.

// The stream is staged in LDS like the parser's payload, in a ring of WRU 16-B units per
// lane (dword k of lane l at ((k mod 4 WRU) * 64 + l) * 4: every lane's read hits bank l):
// a group issues the loads of up to WNL next units at its start and writes them at its end,
// so a load has a group's time to arrive and the window's refills read LDS (a register
// queue of global loads left each load's latency on the word after it: 31.4 ms for C4).
constexpr uint32_t WRU = 8, WNL = 4;
constexpr uint32_t WRING_BYTES = WRU * 16u * 64u;
constexpr uint32_t WRING_OFF = LPAIRS * RING_BYTES + LDS_AFTER_RINGS;  // (HY == 2 kernels: lane_blocks)
__device__ __forceinline__ uint32_t cw_addr(const CWin &c, uint32_t k) { return c.col + ((k & (WRU * 4u - 1u)) << 8); }
__device__ __forceinline__ void cw_put(CWin &c, uint32_t u, uint4 v) {
    uint32_t *d = (uint32_t *)(c.lds + cw_addr(c, 4u * u));  // (the unit's four dwords: consecutive slots)
    d[0] = v.x;
    d[64] = v.y;
    d[128] = v.z;
    d[192] = v.w;
}
__device__ __forceinline__ void cwin_init(CWin &c, const uint8_t *blob, uint8_t *lds, uint32_t pair, uint32_t lane,
                                          uint64_t off, uint32_t len) {
    const uint32_t skip = (uint32_t)(off & 15u);
    c.src = (const uint4 *)(blob + (off - skip));
    c.lds = lds;
    c.col = WRING_OFF + pair * WRING_BYTES + lane * 4u;
    const uint32_t eu = (skip + len + 15u) >> 4;
    c.ulast = eu > 0u ? eu - 1u : 0u;
#pragma unroll
    for (uint32_t u = 0; u < WRU; u++) cw_put(c, u, c.src[min(u, c.ulast)]);
    c.lu = WRU;
    c.lim = 4u * WRU;
    c.ovf = 0u;
    const uint32_t k = skip >> 2, sb = (skip & 3u) * 8u;
    c.win = ((uint64_t)*(const uint32_t *)(c.lds + cw_addr(c, k)) |
             ((uint64_t)*(const uint32_t *)(c.lds + cw_addr(c, k + 1u)) << 32)) >> sb;
    c.nb = 64 - (int32_t)sb;
    c.rd = k + 2u;
    c.nxt = *(const uint32_t *)(c.lds + cw_addr(c, c.rd));
    c.used = 0;
    c.end = len * 8u;
}
// keep >= 33 bits: merge the dword read ahead when 32 or fewer are left, then read the next
__device__ __forceinline__ void cwin_merge(CWin &c) {
    const uint32_t mg = (uint32_t)((c.nb - 33) >> 31);  // ~0: merge
    const uint32_t sh = (uint32_t)c.nb;
    __builtin_assume(sh < 64u);
    c.win |= (uint64_t)(c.nxt & mg) << sh;
    c.nb += (int32_t)(mg & 32u);
    c.ovf |= mg & (c.rd >= c.lim ? 1u : 0u);
    c.rd += mg & 1u;
    c.nxt = *(const uint32_t *)(c.lds + cw_addr(c, c.rd));
}
// a group's staging: the loads of the units after lu that fit in the ring (the dwords
// below rd are merged), issued at the group's start ...
struct CStage {
    uint4 v0, v1, v2, v3;
    uint32_t n;
};
__device__ __forceinline__ CStage cwin_issue(CWin &c) {
    CStage st;
    c.lim = 4u * c.lu;
    const uint32_t room = (c.rd >> 2) + WRU - c.lu;
    st.n = room < WNL ? room : WNL;
    st.v0 = c.src[min(c.lu, c.ulast)];
    st.v1 = c.src[min(c.lu + 1u, c.ulast)];
    st.v2 = c.src[min(c.lu + 2u, c.ulast)];
    st.v3 = c.src[min(c.lu + 3u, c.ulast)];
    return st;
}
// ... and written at its end (a unit without room to the dummy slots past the rings)
__device__ __forceinline__ void cwin_stage(CWin &c, const CStage &st, uint32_t lane) {
    const uint32_t dummy = RING_DUMMY + lane * 4u;
    CWin d = c;
    d.col = dummy;  // (cw_addr of a dummy: its 4 slots of 64 lanes at RING_DUMMY)
    if (st.n > 0u) cw_put(c, c.lu, st.v0); else cw_put(d, 0u, st.v0);
    if (st.n > 1u) cw_put(c, c.lu + 1u, st.v1); else cw_put(d, 0u, st.v1);
    if (st.n > 2u) cw_put(c, c.lu + 2u, st.v2); else cw_put(d, 0u, st.v2);
    if (st.n > 3u) cw_put(c, c.lu + 3u, st.v3); else cw_put(d, 0u, st.v3);
    c.lu += st.n;
}
// exact - lossy for a word of value v (sign and lossy magnitude) whose final interval
// is [lo, lo + n - 1] (n 1: the word was exact, nothing is read, lo its magnitude)
__device__ __forceinline__ int32_t cwin_corr(CWin &c, int32_t v, uint32_t lo, uint32_t n) {
    const int32_t sg = v >> 31;
    const uint32_t mid = (uint32_t)(v ^ sg);
    const uint32_t mc = n - 1u;  // high - low
    const uint32_t x = (uint32_t)c.win;
    const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
    const uint32_t ex = (0xFFFFFFFFu >> z) - mc;
    const uint32_t nbt = z ^ 31u;
    const uint32_t vv = __builtin_amdgcn_ubfe(x, 0, nbt);
    const bool big = vv >= ex;
    const uint32_t code = big ? 2u * vv + __builtin_amdgcn_ubfe(x, nbt, 1) - ex : vv;
    const uint32_t used = nbt + (big ? 1u : 0u);  // (0 for n == 1)
    c.win >>= used;
    c.nb -= (int32_t)used;
    c.used += used;
    cwin_merge(c);
    const uint32_t value = lo + code;
    return (int32_t)(sg ? mid - value : value - mid);
}
// slow_level after a word (HYBRID_BITRATE, :501-502): slow - (slow + SLO) >> SLS + mylog2(mid)
// (mylog2, WordsUtils.cs:588-608: the 8 bits below the leading one index the table)
__device__ __forceinline__ int32_t lhy_slow(int32_t slow, uint32_t mid, const uint8_t *ring) {
    using namespace wvf;
    const uint32_t a = mid + (mid >> 9);
    const uint32_t cz = (uint32_t)__clz((int32_t)a);  // 32 for 0
    const uint32_t idx = ((a << (cz & 31u)) >> 23) & 0xFFu;
    const int32_t lg = (int32_t)(((32u - cz) << 8) + (uint32_t)ring[TAB_LOG2 + idx]);
    return add32(sub32(slow, add32(slow, SLO) >> SLS), lg);
}
__device__ __forceinline__ int32_t lhy_decay(int32_t slow) {  // a zero-run zero's slow_level (:316-317)
    using namespace wvf;
    return sub32(slow, add32(slow, SLO) >> SLS);
}

// A word's result: its value v, and what the reconstruction wave needs to compute it
// itself (CODES, lane_blocks): x, the 32 window bits after the unary part, the bucket's
// low and high - low (mc).  v = (low + read_code(mc) from x) ^ (its sign bit) (rdecode);
// a zero word is x = low = mc = 0, which decodes to 0.
struct LW {
    uint32_t x, low, mc;
    int32_t v;
    uint32_t clo, cn;  // HY == 2: the final interval [clo, clo + cn - 1] of an inexact hybrid word (cn 1: exact)
};

// get_words for one residual of channel C (WordsUtils.cs:290-503, lossless:
// error_limit 0): the word as branch-free selects on lane masks.  Two rare
// parts branch, taken when some lane needs them: the zero-run mode's entry (a
// run length read) and the LIMIT_ONES escape (both refill the window between
// their parts).  Checks are accumulated, not branched on: s.pmax (17: a bits
// error or a count too long for the lane) and s.slack (bits left in the window
// after a part: negative means a word past the window).  A lane inside a zero
// run (zskip) runs the word as a held zero over all-zero medians that consumes
// nothing, which leaves its state as it was -- and the checks it feeds are those
// of the word that ends the run, which reads the same window with the same state.
template <int C, int HY = false>
__device__ __forceinline__ LW lword(LState &s, const uint8_t *ring, uint32_t rbase) {
    using namespace wvf;
    // zero-run mode (:304-352): both channels' median[0] < 2, nothing held
    const uint64_t h0m0 = lmask(s.keep == 0u), h1m0 = lmask(s.h1 != 0u);
    const uint64_t zrm = lmask((((uint32_t)(s.m[0][0] | s.m[1][0])) & ~1u) == 0u) & ~(h0m0 | h1m0);
    bool zskip = false;
    if (__builtin_expect(zrm != 0ull, 0)) {
        if (__builtin_amdgcn_inverse_ballot_w64(zrm)) {
            if (s.zacc > 0u) {
                s.zacc--;
                zskip = s.zacc > 0u;
            } else {
                s.zacc = lgamma(s, ring, rbase);
                if (s.zacc > 0u) {
                    s.m[0][0] = s.m[0][1] = s.m[0][2] = 0;
                    s.m[1][0] = s.m[1][1] = s.m[1][2] = 0;
                    zskip = true;
                }
            }
        }
    }
    const uint64_t zm = lmask(zskip);
    const uint64_t hzm = h0m0 | zm;
    if constexpr (HY) {
        s.slow[C] = zskip ? lhy_decay(s.slow[C]) : s.slow[C];
        if constexpr (C == 0) lhy_errlim(s, ring, !zskip);
    }
    // unary count (:354-428): raw ones (capped at 16) and the bits they take
    const uint32_t lo = (uint32_t)s.win;
    uint32_t raw = (uint32_t)__builtin_ctz(~lo | 0x10000u);
    uint32_t p = raw + 1u;
    const uint64_t escm = lmask(raw >= 16u) & ~hzm;
    if (__builtin_expect(escm != 0ull, 0)) {
        if (__builtin_amdgcn_inverse_ballot_w64(escm)) {
            // 16 ones and a zero, then the escaped count (17 ones: the reference's bits error)
            if (lo & 0x10000u) s.pmax = 17u;
            lskip(s, 17u);
            lrefill(s, ring, rbase);
            raw = lgamma(s, ring, rbase) + 16u;
            if (raw >= (1u << 24)) s.pmax = 17u;  // (ones - 2) stays a 24-bit operand of the bucket product
            p = 0u;
        }
    }
    p = vselm(hzm, 0u, p);
    lskip(s, p);
    lrefill(s, ring, rbase);  // (the code after up to 17 unary bits: up to 26 more bits)
    const uint32_t ones = vselm(hzm, 0u, addc(raw >> 1, h1m0));
    const uint64_t b0m = lmask((raw & 1u) != 0u);
    s.h1 = lbit(~hzm & b0m) ? 1u : 0u;
    s.keep = lbit(~hzm & ~b0m) ? 0u : ~0u;
    const int32_t m0 = s.m[C][0], m1 = s.m[C][1], m2 = s.m[C][2];
    const uint32_t a0 = (uint32_t)(m0 >> 4), a1 = (uint32_t)(m1 >> 4), a2 = (uint32_t)(m2 >> 4);
    const uint64_t o0 = lmask(ones == 0u), o1 = lmask(ones == 1u), o2 = lmask(ones == 2u), ob = o0 | o1;
    const uint32_t mc = vselm(o0, a0, vselm(o1, a1, a2));
    const uint32_t low1 = a0 + 1u;
    // (32-bit products, C#'s int wrap: this word also serves groups whose medians
    // are past the fast words' 24-bit operands)
    const uint32_t low2 = (ones > 2u ? ones - 2u : 0u) * (a2 + 1u) + low1 + a1 + 1u;
    const uint32_t low = vselm(o0, 0u, vselm(o1, low1, low2));
    // median updates (:433-475; DIV0/1/2 as shifts): m + ((m + off) >> s) * mult with
    // (off, mult) = (D - 2, -2) for the bucket's own median, (D, 5) below it, (-, 0) above
    s.m[C][0] = add32(m0, mul32((int32_t)(add3((uint32_t)m0, 128u, (uint32_t)csel<-2, 0>(o0))) >> 7, csel<-2, 5>(o0)));
    s.m[C][1] = add32(m1, mul32((int32_t)(add3((uint32_t)m1, 64u, (uint32_t)csel<-2, 0>(o1))) >> 6,
                                vselmi(o0, 0, csel<-2, 5>(o1))));
    s.m[C][2] = add32(m2, mul32((int32_t)(add3((uint32_t)m2, 32u, (uint32_t)csel<-2, 0>(o2))) >> 5,
                                vselmi(ob, 0, csel<-2, 5>(o2))));
    // read_code(high - low = mc) (WordsUtils.cs:546-570), then the sign bit
    const uint32_t x = (uint32_t)s.win;
    uint32_t mid, used, lo_f = 0u, n_f = 1u;
    if constexpr (HY) {
        lhy_code<HY>(x, low, mc, s.el[C], mid, used, s.bad, lo_f, n_f);
        s.slack = min(s.slack, 31 - (int32_t)used);  // (the sign must lie in x)
    } else {
        const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
        const uint32_t ones_z = 0xFFFFFFFFu >> z;
        const uint32_t ex = ones_z - mc;
        const uint32_t nbt = z ^ 31u;
        const uint32_t v = x & (ones_z >> 1);
        const uint64_t bigm = lmask(v >= ex);
        const uint32_t code = vselm(bigm, 2u * v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex, v);
        used = addc(nbt, bigm);
        mid = low + code;
    }
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)x, used, 1);  // 0 or -1
    lskip(s, vselm(zm, 0u, used + 1u));
    LW w;
    w.v = (int32_t)vselm(zm, 0u, mid ^ (uint32_t)sg);
    w.x = vselm(zm, 0u, x);
    w.low = vselm(zm, 0u, low);
    w.mc = vselm(zm, 0u, mc);
    w.clo = vselm(zm, 0u, mid);
    w.cn = 1u;
    if constexpr (HY == 2) {
        const bool inexact = !zskip && s.el[C] != 0;
        w.clo = inexact ? lo_f : w.clo;
        w.cn = inexact ? n_f : 1u;
    }
    if constexpr (HY) s.slow[C] = zskip ? s.slow[C] : lhy_slow(s.slow[C], mid, ring);
    lrefill(s, ring, rbase);
    return w;
}

// The fast word: lword without its two rare branches, VALU only.  A lane inside
// a zero run counts it down (zskip); a word that would read a run length or an
// escaped unary count only sets s.rare, and the group it is in is decoded again
// from its starting state by lword (lane_parser).
template <int C>
__device__ __forceinline__ LW lword_fast(LState &s, const uint8_t *ring, uint32_t rbase) {
    using namespace wvf;
    // zero-run mode (:304-352): a pending run counts down; its entry is rare.  All
    // as 0/1 lane values (a compound condition would go through SALU mask logic)
    const uint32_t zx = (((uint32_t)(s.m[0][0] | s.m[1][0])) & ~1u) | (s.keep + 1u) | s.h1;
    const uint32_t zrv = zx == 0u ? 1u : 0u;       // the zero-run test holds
    const uint32_t zdec = min(s.zacc, zrv);        // a pending run counts down
    s.zacc -= zdec;
    const uint32_t zsk = min(s.zacc, zdec);        // ... and this word is one of its zeros
    const uint32_t lo = (uint32_t)s.win;
    const uint32_t raw = (uint32_t)__builtin_ctz(~lo | 0x10000u);  // unary ones, capped at 16
    const uint32_t keep = s.keep & (zsk - 1u);    // ~0 for a word that reads its unary count, 0 for a held zero
    const uint32_t p = (raw + 1u) & keep;
    // rare: 16 ones (LIMIT_ONES escape or a bits error: p == 17), or a run length to read
    s.rare |= ((p + 15u) >> 5) | (zrv & (zdec ^ 1u));
    const uint32_t ones = ((raw >> 1) + s.h1) & keep;
    const uint32_t nh1 = raw & 1u & keep;
    s.h1 = nh1;
    s.keep = (uint32_t)__builtin_amdgcn_sbfe((int32_t)(nh1 | ~keep), 0, 1);  // a zero is held after an even count
    s.win >>= p;
    s.nb -= (int32_t)p;
    const int32_t m0 = s.m[C][0], m1 = s.m[C][1], m2 = s.m[C][2];
    const uint32_t a0 = (uint32_t)(m0 >> 4), a1 = (uint32_t)(m1 >> 4), a2 = (uint32_t)(m2 >> 4);
    const bool o0 = ones == 0u, o1 = ones == 1u, o2 = ones == 2u, ob = ones < 2u;
    const uint32_t mc = o0 ? a0 : (o1 ? a1 : a2);
    const uint32_t low1 = a0 + 1u;
    const uint32_t low2 = __umul24(ones > 2u ? ones - 2u : 0u, a2 + 1u) + low1 + a1 + 1u;
    const uint32_t low = o0 ? 0u : (o1 ? low1 : low2);
    // median updates (:433-475), as in lword
    s.m[C][0] = mad24((add32(m0, o0 ? 126 : 128)) >> 7, o0 ? -2 : 5, m0);
    s.m[C][1] = mad24((add32(m1, o1 ? 62 : 64)) >> 6, o0 ? 0 : (o1 ? -2 : 5), m1);
    s.m[C][2] = mad24((add32(m2, o2 ? 30 : 32)) >> 5, ob ? 0 : (o2 ? -2 : 5), m2);
    // read_code(high - low = mc), then the sign bit
    const uint32_t x = (uint32_t)s.win;
    const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
    const uint32_t ones_z = 0xFFFFFFFFu >> z;
    const uint32_t ex = ones_z - mc;
    const uint32_t nbt = z ^ 31u;
    const uint32_t v = x & (ones_z >> 1);
    const bool big = v >= ex;
    const uint32_t code = big ? 2u * v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex : v;
    const uint32_t used = nbt + (big ? 1u : 0u);
    const uint32_t mid = low + code;
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)x, used, 1);  // 0 or -1
    const uint32_t len = (used + 1u) & (zsk - 1u);
    s.win >>= len;
    s.nb -= (int32_t)len;
    s.slack = min(s.slack, s.nb);
    LW w;
    w.v = (int32_t)((mid ^ (uint32_t)sg) & (zsk - 1u));
    w.x = x & (zsk - 1u);
    w.low = low & (zsk - 1u);
    w.mc = mc & (zsk - 1u);
    w.clo = 0u;
    w.cn = 1u;
    lrefill(s, ring, rbase);
    return w;
}

// The no-run word: lword_fast for a group in which no lane can enter the zero-run
// mode (lane_parser checks, per group, that max(median[0] of both channels) >= 18:
// a median[0] falls by at most 2 per word while it is below 130, so the test
// (:304-306, both channels' median[0] < 2) cannot hold in the group's 8 words per
// channel, and no run is pending).  Per word, in issue order of need:
//   unary count raw <= 16 (16: the LIMIT_ONES escape, left to the checked word via
//   s.rmax); a held zero reads no unary bits (raw & keep); q = the unary bits taken;
//   the bucket's medians and bounds (:433-475) as selects; read_code (:546-570) on
//   the 32 bits after the unary part (x, one v_alignbit from the 64-bit window); the
//   word's total length taken from the window once; the refill merges the dword
//   read ahead when 32 bits or fewer are left.
// merge the dword read ahead when 32 bits or fewer are left (and read the next)
__device__ __forceinline__ void lmerge(LState &s, const uint8_t *ring) {
    const uint32_t mg = (uint32_t)((s.nb - 33) >> 31);  // ~0: merge
    const uint32_t sh = (uint32_t)s.nb;
    __builtin_assume(sh < 64u);
    s.win |= (uint64_t)(s.nxt & mg) << sh;
    s.nb = mad24((int32_t)mg, -32, s.nb);
    s.ra = ring_step(s.ra, mg);
    s.nxt = *(const uint32_t *)(ring + s.ra);
}
// SPLIT: the window is refilled between the unary part and the code instead of
// after the word, for groups whose medians allow codes longer than the 33 bits a
// word may count on otherwise (pgroup_try): the code and sign then have >= 33 bits,
// and the next word's unary part whatever is left (>= 1 bit; a unary count that runs
// past it shows as slack < 0, and the group is replayed by the checked words)
// W32: 32-bit products (C#'s int wrap) for groups whose medians pass the 24-bit
// operands (pgroup_try: below 2^29 at the group's start, so none wraps in the group)
// SPEC (the plain no-run word): the next word's unary count is taken before this
// word's refill.  E = the window with the read-ahead dword placed at nb (its low 64
// bits; nb >= 33 at a word start, so only E's high half changes) holds stream bits
// [0, 64) exactly, and the next word's unary bits [tot, tot + 17) lie in it whether
// the refill merges or not (tot <= 47); so s.r0 = ctz over E >> tot, and the
// refill (compare, mask, 64-bit shift, or) leaves the word-to-word chain.
#ifndef WV_LANE_SPEC
#define WV_LANE_SPEC 0
#endif
template <int C, bool SPLIT, int HY = false, bool W32 = false>
__device__ __forceinline__ LW lword_nz(LState &s, const uint8_t *ring, uint32_t rbase) {
    static_assert(!HY || SPLIT, "a hybrid word's bisection bits follow a refill");
    using namespace wvf;
    constexpr bool SPEC = WV_LANE_SPEC && !SPLIT && !HY && !W32;
    const uint32_t lo = (uint32_t)s.win, hi = (uint32_t)(s.win >> 32);
    // unary ones, capped at 16
    const uint32_t raw0 = SPEC ? s.r0 : (uint32_t)__builtin_ctz(~lo | 0x10000u);
    uint32_t ehi = 0u;
    if constexpr (SPEC) {
        const uint32_t sft = (uint32_t)(s.nb - 32) & 63u;  // 1..32 at a word start
        ehi = hi | (uint32_t)((uint64_t)s.nxt << sft);
    }
    s.rmax = max(s.rmax, raw0);
    const uint32_t raw = raw0 & s.keep;          // a held zero: no unary count (ones 0, holding_one clear)
    const uint32_t ones = (raw >> 1) + s.h1;
    const uint32_t q = raw - s.keep;             // unary bits taken: raw + 1, or 0 for a held zero
    s.h1 = raw & 1u;
    s.keep = (uint32_t)__builtin_amdgcn_sbfe((int32_t)(raw | ~s.keep), 0, 1);  // an even count holds a zero
    if constexpr (HY && C == 0) lhy_errlim(s, ring, true);
    const int32_t m0 = s.m[C][0], m1 = s.m[C][1], m2 = s.m[C][2];
    const uint32_t a0 = (uint32_t)(m0 >> 4), a1 = (uint32_t)(m1 >> 4), a2 = (uint32_t)(m2 >> 4);
    const bool o0 = ones == 0u, o1 = ones == 1u;
    const uint32_t mc = o0 ? a0 : (o1 ? a1 : a2);
    // (low as selects of values computed unconditionally: a conditional multiply
    // becomes a divergent branch)
    const uint32_t l3 = (W32 ? (ones > 2u ? ones - 2u : 0u) * (a2 + 1u) : mul_u24(ones > 2u ? ones - 2u : 0u, a2 + 1u)) +
                        a1 + 1u;
    const uint32_t low = vselm(lmask(o0), 0u, add3(a0, 1u, vselm(lmask(o1), 0u, l3)));
    // median k moves by ((m + DIVk + adj) >> sk) * mult: mult 5 above the bucket, -2 in it
    // (adj -2), 0 below; both read from nibble tables at the bucket index min(ones, 3)
    const uint32_t k4 = min(ones, 3u) << 2;
    const int32_t d0 = (int32_t)add3((uint32_t)m0, 128u, (uint32_t)__builtin_amdgcn_sbfe(0x000E, k4, 4)) >> 7;
    const int32_t d1 = (int32_t)add3((uint32_t)m1, 64u, (uint32_t)__builtin_amdgcn_sbfe(0x00E0, k4, 4)) >> 6;
    const int32_t d2 = (int32_t)add3((uint32_t)m2, 32u, (uint32_t)__builtin_amdgcn_sbfe(0x0E00, k4, 4)) >> 5;
    const int32_t x0 = __builtin_amdgcn_sbfe(0x555E, k4, 4), x1 = __builtin_amdgcn_sbfe(0x55E0, k4, 4);
    const int32_t x2 = __builtin_amdgcn_sbfe(0x5E00, k4, 4);
    if constexpr (W32) {
        s.m[C][0] = wvf::add32(m0, wvf::mul32(d0, x0));
        s.m[C][1] = wvf::add32(m1, wvf::mul32(d1, x1));
        s.m[C][2] = wvf::add32(m2, wvf::mul32(d2, x2));
    } else {
        s.m[C][0] = mad24(d0, x0, m0);
        s.m[C][1] = mad24(d1, x1, m1);
        s.m[C][2] = mad24(d2, x2, m2);
    }
    // read_code(mc): nbt = bitcount - 1 bits, one more when v >= extras
    uint32_t x;
    if constexpr (SPLIT) {
        __builtin_assume(q < 64u);
        s.win >>= q;
        s.nb -= (int32_t)q;
        s.slack = min(s.slack, s.nb);
        lmerge(s, ring);
        x = (uint32_t)s.win;
    } else {
        x = __builtin_amdgcn_alignbit(hi, lo, q);
    }
    uint32_t mid, used, lo_f = 0u, n_f = 1u;
    if constexpr (HY) {
        lhy_code<HY>(x, low, mc, s.el[C], mid, used, s.bad, lo_f, n_f);
        s.slack = min(s.slack, 31 - (int32_t)used);  // (the sign must lie in x)
    } else {
        const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
        const uint32_t ex = (0xFFFFFFFFu >> z) - mc;
        const uint32_t nbt = z ^ 31u;
        const uint32_t v = __builtin_amdgcn_ubfe(x, 0, nbt);
        const bool big = v >= ex;
        const uint32_t t = v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex;  // code = v + t when big
        mid = add3(low, v, big ? t : 0u);
        used = nbt + (big ? 1u : 0u);
    }
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)x, used, 1);  // 0 or -1
    const uint32_t tot = SPLIT ? used + 1u : add3(q, used, 1u);
    __builtin_assume(tot < 64u);
    if constexpr (SPEC) s.r0 = (uint32_t)__builtin_ctz(~(uint32_t)((((uint64_t)ehi << 32) | lo) >> tot) | 0x10000u);
    s.win >>= tot;
    s.nb -= (int32_t)tot;
    s.slack = min(s.slack, s.nb);
    if constexpr (!SPLIT) lmerge(s, ring);
    if constexpr (HY) s.slow[C] = lhy_slow(s.slow[C], mid, ring);
#ifdef WV_LANE_WORD_BARRIER  // (experiment: words in program order, the ring read a word ahead of its use)
    __builtin_amdgcn_sched_barrier(WV_LANE_WORD_BARRIER);
#endif
    uint32_t clo = mid, cn = 1u;
    if constexpr (HY == 2) {
        clo = s.el[C] != 0 ? lo_f : mid;
        cn = s.el[C] != 0 ? n_f : 1u;
    }
    return LW{x, low, mc, (int32_t)(mid ^ (uint32_t)sg), clo, cn};
}

// ---------------------------------------------------------------------------
// Two waves per 64 blocks: the PARSER wave runs the words (lword) and hands each
// frame's two residuals to the RECON wave through an LDS ring (RF frames per
// lane); the recon wave runs the passes, joint stereo, the mute bound, the CRC,
// the fixup shift and the stores.  They sit on different SIMDs, so a block's
// critical path is its words alone.  The waves agree through two LDS counters
// (frames produced / consumed, published per group of GF frames) with bounded
// waits: a wait that runs out hands every block of the pair to the two-wave
// kernel (ST_REDO).
// ---------------------------------------------------------------------------
constexpr int RF = 24;                     // frames in flight per lane (parser -> recon): three groups
static_assert(RF % GF == 0, "a group's frames never wrap the frame ring");
constexpr uint32_t LSPIN = 1u << 24;       // bounded waits (polls)

struct LShared {
    // parser -> recon, frame t at [(t % RF) * 64 + lane]: CODES, (x, low) of both words in
    // rq and (mc, mc) in rm; else the two residuals in rm
    int4 rq[RF * 64];
    int2 rm[RF * 64];
    uint32_t pflag[64];                    // parser -> recon: the block's parse verdict (bit 31: final)
    uint32_t produced, consumed, abort;    // frames; abort: a wait ran out
    // (wv_pcm_lane_rt3: reconstruction role h -> h + 1 through ring h, int2 slots in the free
    // rq region: frames handed on / taken; role h's weight verdicts per lane)
    uint32_t hop_out[3], hop_in[3];
    uint32_t rbh[2][64];
};

// the index of the stream dword merged next (< 128 advances since the group's start)
__device__ __forceinline__ uint32_t rpos(const LState &s) { return s.rp + (((s.ra0 - s.ra) & RSLOT) >> 8); }

// the parser's verdict for its lane now (after the block's last frame)
template <int HY>
__device__ __forceinline__ uint32_t pverdict(const LState &s, uint32_t u0) {
    const uint32_t r = s.bad | (s.pmax >= 17u ? 16u : 0u) | (s.slack < 0 ? 32u : 0u) | (rpos(s) >= u0 * 4u ? 64u : 0u);
    return 0x80000000u | r | ((s.bad0 ? s.bad0 : r) << 8);
}

// word kinds: WK_CHECKED lword, WK_FAST lword_fast, WK_NORUN / WK_NORUN_SPLIT lword_nz
enum { WK_CHECKED = 0, WK_FAST = 1, WK_NORUN = 2, WK_NORUN_SPLIT = 3, WK_NORUN_SPLIT32 = 4 };
template <int K, int C, int HY>
__device__ __forceinline__ LW lword_k(LState &s, const uint8_t *ring, uint32_t rb) {
    if constexpr (K == WK_NORUN) return lword_nz<C, false, false>(s, ring, rb);  // (not HY: pgroup_try)
    else if constexpr (K == WK_NORUN_SPLIT) return lword_nz<C, true, HY>(s, ring, rb);
    else if constexpr (K == WK_NORUN_SPLIT32) return lword_nz<C, true, HY, true>(s, ring, rb);
    else if constexpr (K == WK_FAST) return lword_fast<C>(s, ring, rb);
    else return lword<C, HY>(s, ring, rb);
}
template <int U, bool FULL, int FAST, bool MONO, int HY, bool CODES>
__device__ __forceinline__ void pframe(LState &s, const uint8_t *ring, uint32_t rb, LShared &sh, uint32_t lane,
                                       uint32_t g0, uint32_t nfr, uint32_t u0, uint32_t &pfin) {
    const uint32_t t = g0 + U;
    const uint32_t slot = (((g0 % (uint32_t)RF) + U) << 6) + lane;  // (GF divides RF: no wrap inside a group)
    const LW w0 = lword_k<FAST, 0, HY>(s, ring, rb);
    LW w1 = {0u, 0u, 0u, 0, 0u, 1u};
    if constexpr (!MONO) w1 = lword_k<FAST, 1, HY>(s, ring, rb);
    if constexpr (CODES) {
        sh.rq[slot] = make_int4((int32_t)w0.x, (int32_t)w0.low, (int32_t)w1.x, (int32_t)w1.low);
        sh.rm[slot] = make_int2((int32_t)w0.mc, (int32_t)w1.mc);
    } else {
        sh.rm[slot] = make_int2(w0.v, w1.v);
        if constexpr (HY == 2)  // (rq is free without CODES)
            sh.rq[slot] = make_int4((int32_t)w0.clo, (int32_t)w0.cn, (int32_t)w1.clo, (int32_t)w1.cn);
    }
    if (!FULL && t + 1u == nfr) pfin = pverdict<HY>(s, u0);
}
template <bool FULL, int FAST, bool MONO, int HY, bool CODES>
__device__ __forceinline__ void pgroup(LState &s, const uint8_t *ring, uint32_t rb, LShared &sh, uint32_t lane,
                                       uint32_t g0, uint32_t nfr, uint32_t u0, uint32_t &pfin) {
    pframe<0, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<1, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<2, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<3, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<4, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<5, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<6, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
    pframe<7, FULL, FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
}
// a group: the fast words first -- the no-run words when no live lane can meet a
// zero run in it (lword_nz), else lword_fast; if a live lane met a rare word, the
// group again from its starting state with the checked words (the residual slots,
// the ring and the group's loads are untouched by the first attempt's reads)
// The fast words assume every median below 2^26 at the group's start (their
// 24-bit products: a median grows at most 3.2x in a group's 8 words per channel) and
// a window that holds each word (s.slack); a group with a larger median goes to the
// checked words at once (32-bit arithmetic), a fast group that met a longer word is
// decoded again by them (they refill between a word's parts).  mm: the lanes' largest
// median at the group's start.
// (diagnostics, builds with -DWV_LANE_COUNTERS=1) groups per path of one parser wave
// and where its cycles go: wvg_batch_lane_counters.  Off in the product build: each
// test of the counter pointer is a branch per group.
#ifndef WV_LANE_COUNTERS
#define WV_LANE_COUNTERS 0
#endif
#define LCNT(x)                                 \
    do {                                        \
        if constexpr (WV_LANE_COUNTERS != 0) x; \
    } while (0)
struct LCount {
    uint32_t groups, bulk, norun, split, fast, checked, replay;
    uint64_t wait_consumed, wait_loads;  // cycles in the group-start wait and the group-end load wait
    uint64_t words, stage;               // cycles in the group's words (pgroup_try) and in its ring stores
};
template <bool FULL, bool MONO, int HY, bool CODES>
__device__ __forceinline__ void pgroup_try(LState &s, const uint8_t *ring, uint32_t rb, LShared &sh, uint32_t lane,
                                           uint32_t g0, uint32_t nfr, uint32_t u0, uint32_t &pfin, uint32_t mm,
                                           LCount &cnt) {
    LCNT(cnt.groups++);
    // (every wave-wide test below is one compare of a lane value -- a compound
    // condition would go through SALU mask logic, ~20 cycles each way)
    const uint32_t livem = (uint32_t)((int32_t)(g0 - nfr) >> 31);  // ~0: the lane's block has frames left
    s.slack = 0;
    // every live lane inside a zero run for the group's words (:304-316: while the
    // run's count is past 1 a word is a zero that reads nothing and changes no state
    // but the count): one bulk step -- the silence waves (the host's lane order)
    constexpr uint32_t WPG = MONO ? GF : 2 * GF;
    const uint32_t notrun = (((uint32_t)(s.m[0][0] | s.m[1][0])) & ~1u) | ~s.keep | s.h1 | (s.zacc <= WPG ? 1u : 0u);
    if (lmask((notrun & livem) != 0u) == 0ull) {
#pragma unroll
        for (int u = 0; u < GF; u++) {
            const uint32_t slot = (((g0 % (uint32_t)RF) + u) << 6) + lane;
            if constexpr (CODES) sh.rq[slot] = make_int4(0, 0, 0, 0);
            if constexpr (HY == 2) sh.rq[slot] = make_int4(0, 1, 0, 1);
            sh.rm[slot] = make_int2(0, 0);
            if constexpr (HY) {  // every zero of a run decays its channel's slow_level
                s.slow[0] = lhy_decay(s.slow[0]);
                if constexpr (!MONO) s.slow[1] = lhy_decay(s.slow[1]);
            }
        }
        s.zacc -= WPG;
        if (!FULL && livem && nfr <= g0 + GF) pfin = pverdict<HY>(s, u0);
        LCNT(cnt.bulk++);
        return;
    }
    const uint32_t mml = mm & livem;
    const bool m26 = lmask(mml >= (1u << 26)) != 0ull;  // (past the 24-bit products)
    // no lane can meet a zero run in the group: both median[0] >= 18, no run pending
    const uint32_t runnable = ((uint32_t)(max(s.m[0][0], s.m[1][0]) - (2 + 2 * GF)) >> 31) | min(s.zacc, 1u);
#ifndef WV_LANE_HY_PATH  // (diagnostic builds: 1 hybrid groups with large medians, 2 every hybrid group, checked)
#define WV_LANE_HY_PATH 0
#endif
    const bool allnr = lmask((runnable & livem) != 0u) == 0ull &&
                       !(HY && ((WV_LANE_HY_PATH == 1 && m26) || WV_LANE_HY_PATH == 2));
    if (__builtin_expect(m26 && !allnr, 0)) {
        pgroup<FULL, WK_CHECKED, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
        s.bad |= s.slack < 0 ? 32u : 0u;
        LCNT(cnt.checked++);
        return;
    }
    const LState s0 = s;
    const uint32_t pfin0 = pfin;
    if (allnr) {
        // a word may count on 33 bits: 17 of unary count (16 ones are an escape) and a
        // code of 15 + 1 while every median stays below 2^19 -- at most 3.2x its value
        // at the group's start, hence 2^17; with larger medians the window is refilled
        // between a word's parts (a group with a longer word goes to the checked words)
        s.rmax = 0u;
        if (__builtin_expect(m26, 0)) {  // (medians below 2^29, none wraps in the group; or hybrid words)
            pgroup<FULL, WK_NORUN_SPLIT32, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
            lmerge(s, ring);
            LCNT(cnt.split++);
        } else if (!HY && lmask(mml >= (1u << 17)) == 0ull) {
            if constexpr (WV_LANE_SPEC) s.r0 = (uint32_t)__builtin_ctz(~(uint32_t)s.win | 0x10000u);
            pgroup<FULL, WK_NORUN, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
            LCNT(cnt.norun++);
        } else {
            pgroup<FULL, WK_NORUN_SPLIT, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
            lmerge(s, ring);  // (the next group's words start from >= 33 bits)
            LCNT(cnt.split++);
        }
        s.rare = s.rmax >> 4;  // (an escape: the checked words)
    } else if constexpr (HY) {  // (no run-aware fast words for hybrid blocks: the checked words)
        s.slack = 0;
        pgroup<FULL, WK_CHECKED, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
        s.bad |= s.slack < 0 ? 32u : 0u;
        LCNT(cnt.checked++);
        return;
    } else {
        s.rare = 0u;
        pgroup<FULL, WK_FAST, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
        LCNT(cnt.fast++);
    }
    if (__builtin_expect(lmask(((s.rare | ((uint32_t)s.slack >> 31)) & livem) != 0u) != 0ull, 0)) {
        s = s0;
        pfin = pfin0;
        s.slack = 0;
        pgroup<FULL, WK_CHECKED, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin);
        s.bad |= s.slack < 0 ? 32u : 0u;
        LCNT(cnt.replay++);
    }
}

struct LEnd {
    uint32_t *st;
    int32_t ml;
    bool check;      // nframes == block_samples: check_crc_error applies
    int32_t crc;     // the header's crc
    const uint32_t *pflag;
    uint32_t lane;
};
__device__ __forceinline__ void lane_finish(uint32_t rbad, const LEnd &e, int32_t mx, int32_t mn, uint32_t crc) {
    const uint32_t pf = e.pflag[e.lane];
    const uint32_t bad = (rbad | (pf & 0xFFu) | (mx > e.ml || mn < -e.ml ? 8u : 0u));
    uint32_t st = 0;
    if (e.check) {
        st |= ST_CRC_CHECKED;
        if ((int32_t)crc != e.crc) st |= ST_CRC_ERROR;
    }
    *e.st = bad ? (ST_REDO | (bad << 16) | (((pf >> 8) & 0xFFu) << 24)) : st;
}

// a frame's two values (two dword stores: a file's output may start at an odd int)
__device__ __forceinline__ void st2(int32_t *p, int2 v) {
    p[0] = v.x;
    p[1] = v.y;
}

// one frame t = g0 + U of the recon wave.  FULL: every lane of the wave is inside its block.
// MONO: one sample per frame (UnpackUtils.cs:571-588: crc = 3 crc + v), stored once, or
// twice for FALSE_STEREO (fst; :655-664, after the fixup)
// HY: the whole fixup (fixup_tail: float_values, or the lossy clip and shift), else the shift
template <int HY>
__device__ __forceinline__ int32_t lfix(int32_t x, uint32_t sh, const Fixup &fx) {
    if constexpr (HY) return fixup_tail(fx, x);
    else return (int32_t)((uint32_t)x << sh);
}
// a word's value from what the parser passed (LW, CODES): read_code(mc) on x
// (WordsUtils.cs:546-570) plus low, then the sign bit after the code
__device__ __forceinline__ int32_t rdecode(uint32_t x, uint32_t low, uint32_t mc) {
    const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
    const uint32_t ex = (0xFFFFFFFFu >> z) - mc;
    const uint32_t nbt = z ^ 31u;
    const uint32_t v = __builtin_amdgcn_ubfe(x, 0, nbt);
    const bool big = v >= ex;
    const uint32_t t = v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex;  // code = v + t when big
    const uint32_t used = nbt + (big ? 1u : 0u);
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)x, used, 1);
    return (int32_t)(add3(low, v, big ? t : 0u) ^ (uint32_t)sg);
}
// frame t = g0 + U's two word values from the parser's slot
template <int U, bool MONO, bool CODES>
__device__ __forceinline__ void rin(const LShared &shr, uint32_t lane, uint32_t g0, int32_t &L, int32_t &R) {
    const uint32_t slot = (((g0 % (uint32_t)RF) + U) << 6) + lane;
    const int2 r = shr.rm[slot];
    if constexpr (CODES) {
        const int4 q = shr.rq[slot];
        L = rdecode((uint32_t)q.x, (uint32_t)q.y, (uint32_t)r.x);
        R = MONO ? 0 : rdecode((uint32_t)q.z, (uint32_t)q.w, (uint32_t)r.y);
    } else {
        L = r.x;
        R = r.y;
    }
}
// frame t = g0 + U after the passes: joint stereo, the mute bound, the CRC, the fixup,
// the stores, and the block's verdict after its last frame
template <int U, bool FULL, bool MONO, int HY>
__device__ __forceinline__ void rout(int32_t L, int32_t R, uint32_t g0, uint32_t nfr, bool joint, int32_t &mx,
                                     int32_t &mn, uint32_t &crc, uint32_t sh, int32_t *o, uint32_t rbad, const LEnd &e,
                                     bool fst, const Fixup &fx, const CWin &cw) {
    const uint32_t t = g0 + U;
    if constexpr (MONO) {
        mx = max(mx, L);
        mn = min(mn, L);
        crc = crc * 3u + (uint32_t)L;
        const int32_t v = lfix<HY>(L, sh, fx);
        const bool st = FULL ? nfr != 0u : t < nfr;
        if (st) {
            if (fst) st2(o + 2u * t, make_int2(v, v));
            else o[t] = v;
        }
        if (!FULL && t + 1u == nfr) lane_finish(rbad | (HY == 2 && (cw.used > cw.end || cw.ovf) ? 1u : 0u), e, mx, mn, crc);
        return;
    }
    if (joint) {
        R = wvf::sub32(R, L >> 1);
        L = wvf::add32(L, R);
    }
    mx = max(mx, max(L, R));
    mn = min(mn, min(L, R));
    // crc = (crc * 3 + L) * 3 + R (UnpackUtils.cs:620-626)
    crc = crc * 9u + (uint32_t)L * 3u + (uint32_t)R;
    int2 v;
    v.x = lfix<HY>(L, sh, fx);
    v.y = lfix<HY>(R, sh, fx);
    if (FULL) {
        if (nfr) st2(o + 2u * t, v);  // (a lane without a block of its own stores nothing)
    } else {
        if (t < nfr) st2(o + 2u * t, v);
        if (t + 1u == nfr) lane_finish(rbad | (HY == 2 && (cw.used > cw.end || cw.ovf) ? 1u : 0u), e, mx, mn, crc);
    }
}
template <int U, bool FULL, bool MONO, int HY, bool CODES, int... Ts>
__device__ __forceinline__ void rframe(LChain<Ts...> &ch, const LShared &shr, uint32_t lane, uint32_t g0, uint32_t nfr,
                                       bool joint, int32_t &mx, int32_t &mn, uint32_t &crc, uint32_t sh, int32_t *o,
                                       uint32_t rbad, const LEnd &e, bool fst, const Fixup &fx, CWin &cw) {
    const uint32_t t = g0 + U;
    int32_t L, R;
    rin<U, MONO, CODES>(shr, lane, g0, L, R);
    if constexpr (HY == 2) {  // the exact values; the passes keep the lossy history
        const int4 q = shr.rq[(((g0 % (uint32_t)RF) + U) << 6) + lane];
        int32_t cL = 0, cR = 0;
        if (FULL || t < nfr) {  // (a lane past its block reads nothing more)
            cL = cwin_corr(cw, L, (uint32_t)q.x, (uint32_t)q.y);
            cR = cwin_corr(cw, R, (uint32_t)q.z, (uint32_t)q.w);
        }
        ch.template frame_wvc<U, MONO>(L, R, cL, cR);
        L = wvf::add32(L, cL);
        R = wvf::add32(R, cR);
    } else {
        ch.template frame<U, MONO>(L, R);
    }
    rout<U, FULL, MONO, HY>(L, R, g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
}
// a group of a run-time list (RChain): the frames' values, the passes pass-major, the frames' tails
template <bool FULL, bool MONO, bool CODES, int NS, int HY = 0>
__device__ __forceinline__ void rgroup_rt(RChain<NS> &ch, const LShared &shr, uint32_t lane, uint32_t g0, uint32_t nfr,
                                          bool joint, int32_t &mx, int32_t &mn, uint32_t &crc, uint32_t sh, int32_t *o,
                                          uint32_t rbad, const LEnd &e, bool fst, const Fixup &fx, const CWin &cw) {
    int32_t L[GF], R[GF];
    rin<0, MONO, CODES>(shr, lane, g0, L[0], R[0]);
    rin<1, MONO, CODES>(shr, lane, g0, L[1], R[1]);
    rin<2, MONO, CODES>(shr, lane, g0, L[2], R[2]);
    rin<3, MONO, CODES>(shr, lane, g0, L[3], R[3]);
    rin<4, MONO, CODES>(shr, lane, g0, L[4], R[4]);
    rin<5, MONO, CODES>(shr, lane, g0, L[5], R[5]);
    rin<6, MONO, CODES>(shr, lane, g0, L[6], R[6]);
    rin<7, MONO, CODES>(shr, lane, g0, L[7], R[7]);
    ch.template group<MONO>(L, R);
    rout<0, FULL, MONO, HY>(L[0], R[0], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<1, FULL, MONO, HY>(L[1], R[1], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<2, FULL, MONO, HY>(L[2], R[2], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<3, FULL, MONO, HY>(L[3], R[3], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<4, FULL, MONO, HY>(L[4], R[4], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<5, FULL, MONO, HY>(L[5], R[5], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<6, FULL, MONO, HY>(L[6], R[6], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
    rout<7, FULL, MONO, HY>(L[7], R[7], g0, nfr, joint, mx, mn, crc, sh, o, rbad, e, fst, fx, cw);
}

// CODES: the parser hands the reconstruction wave each word's (x, low, mc) and the
// reconstruction computes the value (rdecode), taking ~13 instructions a word off
// the parser's chain -- for term lists whose reconstruction has the room (the 16-term
// lists' passes already load it more than the words load the parser); hybrid words
// (bisection) hand over values
template <int HY, int... Ts>
constexpr bool lane_codes() { return !HY && (LaneRt<Ts...>::NS ? LaneRt<Ts...>::NS : (int)sizeof...(Ts)) <= 5; }

// the lossless lanes' fixup shift (UnpackUtils.cs:1251-1404): the header's, plus an int32
// block's zeros + sent_bits + ones + dups when sent_bits is set (:1344-1345), or its zeros
// alone when it is not (:1327-1330: `<<= zeros` ahead of the header shift; lane_ok keeps
// the two shifts' sum below 32, where the two shifts compose into one)
__device__ __forceinline__ uint32_t lane_shift(const BlockDesc &d) {
    int32_t sh = d.shift;
    if (d.flags & wvf::INT32_DATA)
        sh += d.int32_sent_bits ? d.int32_zeros + d.int32_sent_bits + d.int32_ones + d.int32_dups : d.int32_zeros;
    return (uint32_t)sh & 31u;
}

// can this lane decode block d exactly (else ST_REDO)?
template <bool MONO, int HY, int... Ts>
__device__ __forceinline__ bool lane_ok(const BlockDesc &d) {
    using namespace wvf;
    if (d.kind != KIND_PCM) return false;
    if constexpr (HY == 2) {  // hybrid with its .wvc stream: HYBRID_BITRATE (HYBRID_BALANCE too), not int32
        static_assert(!MONO, "hybrid .wvc lanes: stereo");
        if ((d.flags & (HYBRID_FLAG | HYBRID_BITRATE | INT32_DATA)) != (HYBRID_FLAG | HYBRID_BITRATE)) return false;
    } else if constexpr (HY) {
        // hybrid, with or without HYBRID_BITRATE (and HYBRID_BALANCE); integer, float (float_values)
        // or int32 without a wvx stream (fixup_tail: zeros / ones / dups, or the shift, then the clip)
        if (!(d.flags & HYBRID_FLAG) || (d.wvx_state & 0x100)) return false;
    } else if (d.flags & (HYBRID_FLAG | FLOAT_DATA)) {
        return false;
    } else if (d.flags & INT32_DATA) {
        // lossless int32 without a wvx stream whose fixup is a shift (UnpackUtils.cs:1318-1345:
        // sent_bits, zeros -- which the reference applies before ones / dups -- or none of them;
        // lane_shift); the wvx read and the ones / dups maps go to the two-wave / generic kernels
        if (d.wvx_state & 0x100) return false;
        if (d.int32_sent_bits == 0 && d.int32_zeros == 0 && (d.int32_ones | d.int32_dups) != 0) return false;
        if (d.int32_sent_bits == 0 && d.int32_zeros != 0 && d.int32_zeros + (d.shift & 31) > 31) return false;
    }
    if (((d.flags & MONO_DATA) != 0) != MONO) return false;
    if ((d.wvc_len != 0) != (HY == 2)) return false;  // HY 2: hybrid blocks with their .wvc stream
    if (d.inherit || d.chain_len >= 2 || d.wvx_state || d.xfloat || d.pre_end || d.fstatus) return false;
    if constexpr (LaneRt<Ts...>::NS != 0) {  // a run-time list: its length and terms (lane_block: the pair's list)
        static_assert(HY <= 1, "run-time lists: lossless or hybrid without .wvc");
        if (d.num_terms < 0 || d.num_terms > LaneRt<Ts...>::NS) return false;
        for (int i = 0; i < d.num_terms; i++) {
            const int t = d.term[i];
            // (term 0: pass_stereo's call-position rule, the generic kernel; mono: positive terms)
            if (!((t >= 1 && t <= 8) || t == 17 || t == 18 || (!MONO && t < 0 && t >= -3))) return false;
        }
        return true;
    }
    if (d.num_terms != (int32_t)sizeof...(Ts)) return false;
    constexpr int8_t terms[sizeof...(Ts) + 1] = {(int8_t)Ts..., 0};
    for (int i = 0; i < (int)sizeof...(Ts); i++)
        if (d.term[i] != terms[i]) return false;
    return true;
}

// the per-lane setup both waves share
struct LBlock {
    uint32_t bi, nfr, nmax, nmin;
    bool ok, inl;
    uint32_t tw[4];  // run-time lists: the pair's terms (wave-uniform)
    int32_t nt;
};
template <bool MONO, int HY, int... Ts>
__device__ __forceinline__ LBlock lane_block(const BlockDesc *descs, const uint32_t *list, uint32_t n, uint32_t grp,
                                             uint32_t lane) {
    LBlock b;
    const uint32_t li = grp * 64u + lane;
    // every lane stays in the wave (uniform loops keep the lane masks in SGPRs):
    // a lane past the list or with a block it does not take decodes 0 frames
    b.inl = li < n && list[li] != kLaneGap;
    b.bi = b.inl ? list[li] : 0u;
    b.ok = b.inl && lane_ok<MONO, HY, Ts...>(descs[b.bi]);
    b.tw[0] = b.tw[1] = b.tw[2] = b.tw[3] = 0u;
    b.nt = 0;
    if constexpr (LaneRt<Ts...>::NS != 0) {
        // the pair's list: its first decodable block's; a block with another list is handed back
        // (the host orders the lane list by list, in waves of their own)
        const uint64_t m = lmask(b.ok);
        if (m != 0ull) {
            const uint32_t f = (uint32_t)__builtin_ctzll(m);
            const BlockDesc &d = descs[b.bi];
            const uint32_t *tp = (const uint32_t *)d.term;
            const int32_t nt = d.num_terms;
            b.nt = __builtin_amdgcn_readlane(nt, f);
            bool same = nt == b.nt;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t w = tp[k];
                b.tw[k] = __builtin_amdgcn_readlane(w, f);
                const int32_t nb = min(max(b.nt - 4 * k, 0), 4);  // this dword's bytes inside the list
                const uint32_t bm = nb >= 4 ? ~0u : ((1u << (8 * nb)) - 1u);
                same = same && ((w ^ b.tw[k]) & bm) == 0u;
            }
            b.ok = b.ok && same;
        }
    }
    b.nfr = b.ok ? descs[b.bi].nframes : 0u;
    // the wave runs to its longest block; groups inside every block skip the per-frame end tests
    uint32_t nmax = b.nfr, nmin = b.nfr ? b.nfr : 0xFFFFFFFFu;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off));
        nmin = min(nmin, (uint32_t)__shfl_xor((int)nmin, off));
    }
    b.nmax = __builtin_amdgcn_readfirstlane(nmax);
    b.nmin = __builtin_amdgcn_readfirstlane(nmin);
    return b;
}

// bounded wait until *ctr >= v (or the pair aborted); false when it ran out
__device__ __forceinline__ bool lwait(uint32_t *ctr, uint32_t v, uint32_t *abort_flag) {
    for (uint32_t spins = 0; spins < LSPIN; spins++) {
        if (w2::uni(w2::lds_load_acq(ctr)) >= v) return true;
        if (w2::uni(w2::lds_load_acq(abort_flag))) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    w2::lds_store_rel(abort_flag, 1u);
    return false;
}

template <bool MONO, int HY, int... Ts>
__device__ __forceinline__ void lane_parser(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                            uint32_t n, const uint8_t *__restrict__ blob, LShared &sh,
                                            uint8_t *ringm, uint32_t pair, uint32_t grp, uint32_t lane,
                                            uint32_t *__restrict__ dbg) {
    using namespace wvf;
    constexpr bool CODES = lane_codes<HY, Ts...>();
    const uint64_t t_start = WV_LANE_COUNTERS ? __builtin_readcyclecounter() : 0;
    LCount cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const LBlock lb = lane_block<MONO, HY, Ts...>(descs, list, n, grp, lane);
    const BlockDesc &d = descs[lb.bi];
    const uint32_t nfr = lb.nfr;
    const uint8_t *ring = ringm;
    const uint32_t rb = pair * RING_BYTES + lane * 4u;  // this lane's column of its pair's ring

    // payload: 16-B units from the aligned base; bytes at or past e read 0xFF
    const uint64_t boff = d.bits_off;
    const uint4 *src = (const uint4 *)(blob + (boff & ~(uint64_t)15));
    const uint32_t skip = (uint32_t)(boff & 15u);
    const uint32_t e = lb.ok ? skip + d.bits_len : 0u;
    const uint32_t eu = (e + 15u) >> 4;
    const uint32_t ulast = eu > 0u ? eu - 1u : 0u;
    const uint32_t euk = lb.ok ? eu : 0xFFFFFF00u;  // (the stream-end test as one compare)
    // (units past the stream re-read its last one and read as 0xFF; the 0xFF fill
    // only where some lane's stream ends: a wave-uniform branch)
#pragma unroll 4
    for (uint32_t u = 0; u < (uint32_t)RU; u++) {
        uint4 v = src[min(u, ulast)];
        if (lmask(u + 1u >= euk) != 0ull) v = ff_unit(v, u, e);
        put_unit(ringm, rb, u, v);
    }
    uint32_t fu = RU;  // next unit to load

    LState s;
    s.rp = skip >> 2;
    s.ra = rslot(s.rp) | rb;
    s.win = (uint64_t)(*(const uint32_t *)(ring + s.ra)) |
            ((uint64_t)(*(const uint32_t *)(ring + (rslot(s.rp + 1u) | rb))) << 32);
    s.win >>= (skip & 3u) * 8u;
    s.nb = 64 - (int32_t)((skip & 3u) * 8u);
    s.rp += 2u;
    s.ra = rslot(s.rp) | rb;
    s.ra0 = s.ra;
    s.nxt = *(const uint32_t *)(ring + s.ra);
    s.keep = ~0u;
    s.h1 = 0u;
    s.rare = 0u;
    s.rmax = 0u;
    s.zacc = 0u;
    s.pmax = 0u;
    s.slack = 0;
    s.bad = 0u;
    s.bad0 = 0u;
    s.nobr = (HY && !(d.flags & HYBRID_BITRATE)) ? ~0u : 0u;
    s.bal = (HY && !MONO && (d.flags & HYBRID_BALANCE) && !s.nobr) ? ~0u : 0u;
#pragma unroll
    for (int c = 0; c < 2; c++) {
#pragma unroll
        for (int k = 0; k < 3; k++) s.m[c][k] = d.median[c][k];
        // (set in every instantiation: left undefined, the unused fields of the state
        // copies stay memory, which the backend would place in LDS)
        s.slow[c] = HY ? d.slow_level[c] : 0;
        s.acc[c] = HY ? d.bitrate_acc[c] : 0;
        s.dlt[c] = HY ? d.bitrate_delta[c] : 0;
        s.el[c] = 0;
    }
    // (every field set in every instantiation: left undefined, they stay memory -- scratch)
    uint32_t pfin = 0u;
    uint32_t cpre = 0u;  // the recon's consumed count, read a group ahead (a lower bound: it only grows)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), lgkm/exp untouched: the loop's waits count only its own loads
    for (uint32_t g0 = 0; g0 < lb.nmax; g0 += GF) {
        // the recon wave has taken the frames this group overwrites (RF = 3 groups: the
        // count read at the last group's end nearly always suffices; else wait for it)
        const uint64_t tw0 = (WV_LANE_COUNTERS && dbg) ? __builtin_readcyclecounter() : 0;
        const uint32_t need = g0 + GF > (uint32_t)RF ? g0 + GF - RF : 0u;
        if (w2::uni(cpre) < need && !lwait(&sh.consumed, need, &sh.abort)) return;
        if (WV_LANE_COUNTERS && dbg) cnt.wait_consumed += __builtin_readcyclecounter() - tw0;
        // a bound that keeps the group exact (else the two-wave kernel redoes the block;
        // the reason lands in status bits 16-23 beside ST_REDO, for diagnostics)
        // (unsigned: a median that wrapped negative counts as past every bound)
        const uint32_t u00 = (uint32_t)s.m[0][0], u01 = (uint32_t)s.m[0][1], u02 = (uint32_t)s.m[0][2];
        const uint32_t u10 = (uint32_t)s.m[1][0], u11 = (uint32_t)s.m[1][1], u12 = (uint32_t)s.m[1][2];
        const uint32_t mm = MONO ? max(max(u00, u01), u02) : max(max(max(u00, u01), max(u02, u10)), max(u11, u12));
        // (the checked words' int32 products hold to 2^31; a hybrid word checks its own
        // bounds -- lhy_code: any median, wrapped or not, is exact or handed back)
        if constexpr (!HY) s.bad |= (mm >= (1u << 29) ? 2u : 0u);
        // this group's loads: the units after fu that fit in the ring (four every
        // group, unconditionally: the waitcnt pass then knows exactly which memory
        // operations are in flight; units past the stream re-read its last one)
        const uint32_t u0 = fu;
        const uint32_t room = (s.rp >> 2) + (uint32_t)RU - u0;
        const uint32_t nld = room < (uint32_t)NLD ? room : (uint32_t)NLD;
        uint4 st0 = src[min(u0, ulast)], st1 = src[min(u0 + 1u, ulast)];
        uint4 st2 = src[min(u0 + 2u, ulast)], st3 = src[min(u0 + 3u, ulast)];
        fu = u0 + nld;
        const uint64_t tg0 = (WV_LANE_COUNTERS && dbg) ? __builtin_readcyclecounter() : 0;
        if (g0 + GF < lb.nmin)  // (strict: the group holding a block's last frame records its verdict)
            pgroup_try<true, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin, mm, cnt);
        else
            pgroup_try<false, MONO, HY, CODES>(s, ring, rb, sh, lane, g0, nfr, u0, pfin, mm, cnt);
        if (WV_LANE_COUNTERS && dbg) cnt.words += __builtin_readcyclecounter() - tg0;
        // the reader stayed inside the units written before this group
        s.rp = rpos(s);
        s.ra0 = s.ra;
        if (s.rp >= u0 * 4u) s.bad |= 64u;
        if (!s.bad0) s.bad0 = s.bad | (s.pmax >= 17u ? 16u : 0u);
        // the loads land in the ring (the unit holding the stream end gets its 0xFF tail)
        if (WV_LANE_COUNTERS && dbg) {
            const uint64_t tl0 = __builtin_readcyclecounter();
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            cnt.wait_loads += __builtin_readcyclecounter() - tl0;
        }
        // publish the group: residuals and verdicts first, then the count (before the
        // ring stores, which only this wave reads: the publish waits for no more than
        // the group's residual stores)
        sh.pflag[lane] = pfin;
        w2::lds_publish(&sh.produced, g0 + GF);
        cpre = __hip_atomic_load(&sh.consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t ts0 = (WV_LANE_COUNTERS && dbg) ? __builtin_readcyclecounter() : 0;
        // (branch-free: the 0xFF fill in the groups where some lane's stream ends, a
        // wave-uniform test; a unit without room in the lane's ring to the dummy slots)
        if (lmask(u0 + (uint32_t)NLD >= euk) != 0ull) {
            st0 = ff_unit(st0, u0, e);
            st1 = ff_unit(st1, u0 + 1u, e);
            st2 = ff_unit(st2, u0 + 2u, e);
            st3 = ff_unit(st3, u0 + 3u, e);
        }
        const uint32_t dcol = RING_DUMMY + lane * 4u;
        put_unit_at(ringm, nld > 0u ? unit_addr(rb, u0) : dcol, st0);
        put_unit_at(ringm, nld > 1u ? unit_addr(rb, u0 + 1u) : dcol, st1);
        put_unit_at(ringm, nld > 2u ? unit_addr(rb, u0 + 2u) : dcol, st2);
        put_unit_at(ringm, nld > 3u ? unit_addr(rb, u0 + 3u) : dcol, st3);
        if (WV_LANE_COUNTERS && dbg) cnt.stage += __builtin_readcyclecounter() - ts0;
    }
    if (WV_LANE_COUNTERS && dbg && lane == 0u) {  // (diagnostics: cycles and groups per path of this wave)
        uint32_t *o = dbg + grp * 16u;
        o[0] = (uint32_t)(__builtin_readcyclecounter() - t_start);
        o[1] = cnt.groups;
        o[2] = cnt.bulk;
        o[3] = cnt.norun;
        o[4] = cnt.split;
        o[5] = cnt.fast;
        o[6] = cnt.checked;
        o[7] = cnt.replay;
        o[8] = (uint32_t)cnt.wait_consumed;
        o[9] = (uint32_t)cnt.wait_loads;
        o[10] = (uint32_t)cnt.words;
        o[11] = (uint32_t)cnt.stage;
    }
}

template <bool MONO, int HY, int... Ts>
__device__ __forceinline__ void lane_recon(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                           uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                           uint32_t *__restrict__ status, LShared &sh, uint8_t *lds, uint32_t pair,
                                           uint32_t grp, uint32_t lane) {
    using namespace wvf;
    constexpr bool CODES = lane_codes<HY, Ts...>();
    const LBlock lb = lane_block<MONO, HY, Ts...>(descs, list, n, grp, lane);
    const BlockDesc &d = descs[lb.bi];
    const uint32_t nfr = lb.nfr;
    const bool fst = (d.flags & FALSE_STEREO) != 0;
    if (lb.inl && !lb.ok) status[lb.bi] = ST_REDO | (1u << 16);
    const bool joint = (d.flags & JOINT_STEREO) != 0;
    const uint32_t sh_ = lane_shift(d);
    const int32_t ml = d.mute_limit;
    int32_t *o = out + d.out_off;
    constexpr int NS = LaneRt<Ts...>::NS;
    typename ChainOf<Ts...>::type ch;
    if constexpr (NS != 0) ch.init(d, lb.tw, 0, lb.nt);
    else ch.init(d, 0);
    Fixup fx;
    if constexpr (HY) fixup_init(fx, d);
    // the .wvc stream (HY == 2): this wave reads the corrections -- the parser hands over
    // each word's final interval, off its own chain
    CWin cw;
    if constexpr (HY == 2) cwin_init(cw, blob, lds, pair, lane, lb.ok ? d.wvc_off : 0u, lb.ok ? d.wvc_len : 0u);
    else cw = CWin{nullptr, nullptr, 0u, 0ull, 0, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    uint32_t crc = 0xFFFFFFFFu;
    int32_t mx = 0, mn = 0;
    uint32_t rbad = 0u;
    const LEnd le = {status + lb.bi, ml, d.nframes == d.block_samples, d.crc, sh.pflag, lane};
    __builtin_amdgcn_s_waitcnt(0x0F70);
    for (uint32_t g0 = 0; g0 < lb.nmax; g0 += GF) {
        if (!lwait(&sh.produced, g0 + GF, &sh.abort)) {
            // the parser stopped: every unfinished block of the pair to the two-wave kernel
            if (lb.ok && nfr > g0) status[lb.bi] = ST_REDO | (128u << 16);
            return;
        }
        rbad |= ch.wbad() ? 4u : 0u;
        CStage cst;
        if constexpr (HY == 2) cst = cwin_issue(cw);  // (the next units of the .wvc stream)
        if constexpr (NS != 0) {
            if (g0 + GF < lb.nmin)
                rgroup_rt<true, MONO, CODES, NS, HY>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            else
                rgroup_rt<false, MONO, CODES, NS, HY>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
        } else if (g0 + GF < lb.nmin) {
            rframe<0, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<1, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<2, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<3, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<4, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<5, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<6, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<7, true, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
        } else {
            rframe<0, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<1, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<2, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<3, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<4, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<5, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<6, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
            rframe<7, false, MONO, HY, CODES>(ch, sh, lane, g0, nfr, joint, mx, mn, crc, sh_, o, rbad, le, fst, fx, cw);
        }
        if constexpr (HY == 2) cwin_stage(cw, cst, lane);
        // the group's residuals are read (DS ops of one wave complete in order)
        w2::lds_publish(&sh.consumed, g0 + GF);
    }
    // (every block with frames was finished by lane_finish in its last group)
    if (lb.ok && nfr == 0u)
        status[lb.bi] = (d.block_samples == 0u) ? ST_CRC_CHECKED | ((int32_t)0xFFFFFFFFu != d.crc ? ST_CRC_ERROR : 0u) : 0u;
}

// Run-time lists of 6..16 terms (wv_pcm_lane_rt3): NW reconstruction waves per pair in
// a pipeline -- role r runs its share of the passes and hands each frame on through ring r
// (int2 slots in the rq region, free without CODES), the last role runs the rest and the
// frame tails -- so that each holds at most RS passes' registers and shares its SIMD
// with another chain (lane_blocks_rt3).
template <int NW>
struct RSplit {
#ifndef WV_RT3_RS  // (A/B builds: the passes per role, and the frame tails' weight in passes)
#define WV_RT3_RS 6
#endif
#ifndef WV_RT3_TAILW
#define WV_RT3_TAILW 1
#endif
    static constexpr int RS = NW == 2 ? 8 : WV_RT3_RS;  // passes per role, at most
    static_assert(NW * RS >= MAXP, "the roles cover every list");
    // role r's passes [first, first + count) of nt (the last role also runs the tails: one more share)
    __device__ __forceinline__ static void share(int32_t nt, int role, int32_t &first, int32_t &count) {
        const int32_t q = min((nt + WV_RT3_TAILW + NW - 1) / NW, (int32_t)RS);
        first = min(q * (role - 1), nt);
        count = role < NW ? min(q, nt - first) : nt - first;
    }
};
template <bool MONO>
__device__ __forceinline__ void rin2(const int2 *ring2, uint32_t lane, uint32_t g0, int32_t (&L)[GF], int32_t (&R)[GF]) {
#pragma unroll
    for (int u = 0; u < GF; u++) {
        const int2 r = ring2[(((g0 % (uint32_t)RF) + u) << 6) + lane];
        L[u] = r.x;
        R[u] = MONO ? 0 : r.y;
    }
}
template <bool MONO, int ROLE, int NW, int HY>
__device__ __forceinline__ void lane_recon_split(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                 uint32_t n, int32_t *__restrict__ out, uint32_t *__restrict__ status,
                                                 LShared &sh, uint32_t grp, uint32_t lane) {
    using namespace wvf;
    static_assert(ROLE >= 1 && ROLE <= NW && NW <= 3, "roles");
    const LBlock lb = lane_block<MONO, HY, LANE_RT, 16>(descs, list, n, grp, lane);
    const BlockDesc &d = descs[lb.bi];
    const uint32_t nfr = lb.nfr;
    int32_t first, count;
    RSplit<NW>::share(lb.nt, ROLE, first, count);
    RChain<RSplit<NW>::RS> ch;
    ch.init(d, lb.tw, first, count);
    int2 *const rings2 = (int2 *)sh.rq;  // ring h (1 .. NW - 1) at rings2 + (h - 1) * RF * 64
    static_assert(sizeof(LShared::rq) >= 2 * RF * 64 * sizeof(int2), "two hop rings in rq");
    uint32_t rbad = 0u;
    int32_t L[GF], R[GF];
    if constexpr (ROLE < NW) {
        int2 *const rout2 = rings2 + (ROLE - 1) * RF * 64;
        uint32_t cpre = 0u;  // the next role's consumed count, read a group ahead
        __builtin_amdgcn_s_waitcnt(0x0F70);
        for (uint32_t g0 = 0; g0 < lb.nmax; g0 += GF) {
            if (!lwait(ROLE == 1 ? &sh.produced : &sh.hop_out[ROLE - 1], g0 + GF, &sh.abort)) return;
            const uint32_t need = g0 + GF > (uint32_t)RF ? g0 + GF - RF : 0u;
            if (w2::uni(cpre) < need && !lwait(&sh.hop_in[ROLE], need, &sh.abort)) return;
            rbad |= ch.wbad() ? 4u : 0u;
            if constexpr (ROLE == 1) {
                rin<0, MONO, false>(sh, lane, g0, L[0], R[0]);
                rin<1, MONO, false>(sh, lane, g0, L[1], R[1]);
                rin<2, MONO, false>(sh, lane, g0, L[2], R[2]);
                rin<3, MONO, false>(sh, lane, g0, L[3], R[3]);
                rin<4, MONO, false>(sh, lane, g0, L[4], R[4]);
                rin<5, MONO, false>(sh, lane, g0, L[5], R[5]);
                rin<6, MONO, false>(sh, lane, g0, L[6], R[6]);
                rin<7, MONO, false>(sh, lane, g0, L[7], R[7]);
            } else {
                rin2<MONO>(rings2 + (ROLE - 2) * RF * 64, lane, g0, L, R);
                rbad |= sh.rbh[ROLE - 2][lane];
            }
            ch.template group<MONO>(L, R);
#pragma unroll
            for (int u = 0; u < GF; u++) rout2[(((g0 % (uint32_t)RF) + u) << 6) + lane] = make_int2(L[u], R[u]);
            sh.rbh[ROLE - 1][lane] = rbad;
            // (DS ops of one wave complete in order: the input slots are read, the frames written)
            w2::lds_publish(ROLE == 1 ? &sh.consumed : &sh.hop_in[ROLE - 1], g0 + GF);
            w2::lds_publish(&sh.hop_out[ROLE], g0 + GF);
            cpre = __hip_atomic_load(&sh.hop_in[ROLE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else {
        const bool fst = (d.flags & FALSE_STEREO) != 0;
        if (lb.inl && !lb.ok) status[lb.bi] = ST_REDO | (1u << 16);
        const bool joint = (d.flags & JOINT_STEREO) != 0;
        const uint32_t sh_ = lane_shift(d);
        int32_t *o = out + d.out_off;
        Fixup fx;
        if constexpr (HY) fixup_init(fx, d);
        const CWin cw = CWin{nullptr, nullptr, 0u, 0ull, 0, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        uint32_t crc = 0xFFFFFFFFu;
        int32_t mx = 0, mn = 0;
        const LEnd le = {status + lb.bi, d.mute_limit, d.nframes == d.block_samples, d.crc, sh.pflag, lane};
        __builtin_amdgcn_s_waitcnt(0x0F70);
        for (uint32_t g0 = 0; g0 < lb.nmax; g0 += GF) {
            if (!lwait(&sh.hop_out[NW - 1], g0 + GF, &sh.abort)) {
                if (lb.ok && nfr > g0) status[lb.bi] = ST_REDO | (128u << 16);
                return;
            }
            rbad |= ch.wbad() ? 4u : 0u;
            rin2<MONO>(rings2 + (NW - 2) * RF * 64, lane, g0, L, R);
            const uint32_t rb = rbad | sh.rbh[NW - 2][lane];
            ch.template group<MONO>(L, R);
            if (g0 + GF < lb.nmin) {
                rout<0, true, MONO, HY>(L[0], R[0], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<1, true, MONO, HY>(L[1], R[1], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<2, true, MONO, HY>(L[2], R[2], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<3, true, MONO, HY>(L[3], R[3], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<4, true, MONO, HY>(L[4], R[4], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<5, true, MONO, HY>(L[5], R[5], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<6, true, MONO, HY>(L[6], R[6], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<7, true, MONO, HY>(L[7], R[7], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
            } else {
                rout<0, false, MONO, HY>(L[0], R[0], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<1, false, MONO, HY>(L[1], R[1], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<2, false, MONO, HY>(L[2], R[2], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<3, false, MONO, HY>(L[3], R[3], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<4, false, MONO, HY>(L[4], R[4], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<5, false, MONO, HY>(L[5], R[5], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<6, false, MONO, HY>(L[6], R[6], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
                rout<7, false, MONO, HY>(L[7], R[7], g0, nfr, joint, mx, mn, crc, sh_, o, rb, le, fst, fx, cw);
            }
            w2::lds_publish(&sh.hop_in[NW - 1], g0 + GF);
        }
        if (lb.ok && nfr == 0u)
            status[lb.bi] = (d.block_samples == 0u) ? ST_CRC_CHECKED | ((int32_t)0xFFFFFFFFu != d.crc ? ST_CRC_ERROR : 0u) : 0u;
    }
}

// LPAIRS (parser, recon) wave pairs per workgroup, each pair 64 blocks: the 4 waves
// of a workgroup take the 4 SIMDs of one CU.  Its LDS (2 x ~50 KiB: the 32-unit
// payload rings) is more than half a CU's 160 KiB, so no second workgroup -- of
// this batch or of another in flight -- can land on that CU and put two parser
// waves on one SIMD: measured with 20 batches in flight, 16-unit rings (68 KiB per
// workgroup, two per CU possible) ran at ~30,000 Msamples/s on most runs and
// ~47,000 on some; a workgroup per CU keeps every launch at its one-batch time.
template <bool MONO, int HY, int... Ts>
__device__ __forceinline__ void lane_blocks(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                            uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                            uint32_t *__restrict__ status, uint32_t *__restrict__ dbg) {
    __shared__ LShared shp[LPAIRS];
    // the parsers' payload rings (put_unit, ring_step), the exp2 / log2 tables (HY), the dummy unit
    // slots, and with .wvc streams (HY == 2) the reconstruction waves' correction rings (CWin)
    __shared__ uint32_t rings[(LPAIRS * RING_BYTES + LDS_AFTER_RINGS + (HY == 2 ? LPAIRS * WRING_BYTES : 0u)) / 4];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t pair = wave >> 1, grp = blockIdx.x * LPAIRS + pair;
    LShared &sh = shp[pair];
    if (lane == 0 && (wave & 1u) == 0u) {
        sh.produced = 0u;
        sh.consumed = 0u;
        sh.abort = 0u;
    }
    if constexpr (HY) {
        if (threadIdx.x < 128u) {
            const uint32_t i = threadIdx.x & 63u;
            const auto *tab = (const __attribute__((address_space(4))) uint32_t *)(threadIdx.x < 64u ? c_exp2_table : c_log2_table);
            rings[(threadIdx.x < 64u ? TAB_EXP2 : TAB_LOG2) / 4u + i] = tab[i];
        }
    }
    __syncthreads();
    if (grp * 64u >= n) return;  // (both waves of the pair: uniform)
    if ((wave & 1u) == 0u)
        lane_parser<MONO, HY, Ts...>(descs, list, n, blob, sh, (uint8_t *)rings, pair, grp, lane, dbg);
    else
        lane_recon<MONO, HY, Ts...>(descs, list, n, blob, out, status, sh, (uint8_t *)rings, pair, grp, lane);
}

#ifndef WV_RT_SPLIT16  // (0: A/B builds with every run-time list on the two-wave layout)
#define WV_RT_SPLIT16 1
#endif
// run-time term lists (RChain): each pair takes the variant of its first listed block --
// mono or stereo, up to 5 terms (CODES: the reconstruction computes the word values; longer
// lists: lane_blocks_rt3) -- and the list of its first decodable block (lane_block)
__device__ __forceinline__ void lane_blocks_rt(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                               uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                               uint32_t *__restrict__ status, uint32_t *__restrict__ dbg) {
    __shared__ LShared shp[LPAIRS];
    __shared__ uint32_t rings[(LPAIRS * RING_BYTES + LDS_AFTER_RINGS) / 4];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t pair = wave >> 1, grp = blockIdx.x * LPAIRS + pair;
    LShared &sh = shp[pair];
    if (lane == 0 && (wave & 1u) == 0u) {
        sh.produced = 0u;
        sh.consumed = 0u;
        sh.abort = 0u;
    }
    {   // the exp2 / log2 tables of the hybrid words (a pair of hybrid blocks may come)
        if (threadIdx.x < 128u) {
            const uint32_t i = threadIdx.x & 63u;
            const auto *tab = (const __attribute__((address_space(4))) uint32_t *)(threadIdx.x < 64u ? c_exp2_table : c_log2_table);
            rings[(threadIdx.x < 64u ? TAB_EXP2 : TAB_LOG2) / 4u + i] = tab[i];
        }
    }
    __syncthreads();
    if (grp * 64u >= n) return;  // (both waves of the pair: uniform)
    const uint32_t li = grp * 64u + lane;
    const bool inl = li < n && list[li] != kLaneGap;
    const uint64_t m = lmask(inl);
    if (m == 0ull) return;
    const uint32_t f = (uint32_t)__builtin_ctzll(m);
    const BlockDesc &d0 = descs[inl ? list[li] : 0u];
    const uint32_t fl = __builtin_amdgcn_readlane(d0.flags, f);
    const int32_t nt = __builtin_amdgcn_readlane(d0.num_terms, f);
    uint8_t *rg = (uint8_t *)rings;
    const bool parser = (wave & 1u) == 0u;
#define WV_RT_PAIR(MONO_, NS_, HY_)                                                                  \
    do {                                                                                           \
        if (parser) lane_parser<MONO_, HY_, LANE_RT, NS_>(descs, list, n, blob, sh, rg, pair, grp, lane, dbg); \
        else lane_recon<MONO_, HY_, LANE_RT, NS_>(descs, list, n, blob, out, status, sh, rg, pair, grp, lane); \
    } while (0)
#if WV_RT_SPLIT16  // lists of 6..16 terms: wv_pcm_lane_rt3
    if (nt > 5) return;
    if (fl & wvf::HYBRID_FLAG) {  // (hybrid lanes: HYBRID_BITRATE, lane_ok)
        if (fl & wvf::MONO_DATA) WV_RT_PAIR(true, 5, 1);
        else WV_RT_PAIR(false, 5, 1);
    } else if (fl & wvf::MONO_DATA) {
        WV_RT_PAIR(true, 5, 0);
    } else {
        WV_RT_PAIR(false, 5, 0);
    }
#else  // (A/B builds: every run-time list on one reconstruction wave)
    if (fl & wvf::MONO_DATA) {
        if (nt <= 5) WV_RT_PAIR(true, 5, 0);
        else WV_RT_PAIR(true, 16, 0);
    } else {
        if (nt <= 5) WV_RT_PAIR(false, 5, 0);
        else WV_RT_PAIR(false, 16, 0);
    }
#endif
#undef WV_RT_PAIR
}


// wv_pcm_lane_rt3: the pairs of run-time lists of 6..16 terms (lane_blocks_rt takes the
// others), 1 + RT3_NW waves each -- the parser and RT3_NW reconstruction waves
// (lane_recon_split).  A workgroup's wave w runs on SIMD w % 4; the roles are placed so
// that no SIMD holds two parsers and the reconstruction load spreads: with three
// reconstruction waves, SIMD 0 holds both pairs' first, SIMD 1 both seconds, SIMDs 2 / 3
// a parser each with its pair's last (the lightest: it ends with the tails); with two,
// SIMDs 0 / 1 one pair's two each and SIMDs 2 / 3 the parsers.
#ifndef RT3_NW
#define RT3_NW 3
#endif
constexpr int RT3_THREADS = 64 * (1 + RT3_NW) * LPAIRS;
// (HYK: the lossless pairs (0) or the hybrid ones (1): two kernels, two translation units)
template <int HYK>
__device__ __forceinline__ void lane_blocks_rt3(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                                uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                                uint32_t *__restrict__ status, uint32_t *__restrict__ dbg) {
    static_assert(LPAIRS == 2, "wave roles");
    __shared__ LShared shp[LPAIRS];
    __shared__ uint32_t rings[(LPAIRS * RING_BYTES + LDS_AFTER_RINGS) / 4];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    // (pair, role) of wave w: role 0 the parser, 1..RT3_NW the reconstruction pipeline
#if RT3_NW == 3
    constexpr uint8_t kPair[8] = {0, 0, 0, 1, 1, 1, 0, 1}, kRole[8] = {1, 2, 0, 0, 1, 2, 3, 3};
#else
    constexpr uint8_t kPair[6] = {0, 1, 0, 1, 0, 1}, kRole[6] = {1, 1, 0, 0, 2, 2};
#endif
    const uint32_t role = kRole[wave], pair = kPair[wave], grp = blockIdx.x * LPAIRS + pair;
    LShared &sh = shp[pair];
    if (lane == 0 && role == 0u) {
        sh.produced = 0u;
        sh.consumed = 0u;
        sh.abort = 0u;
#pragma unroll
        for (int h = 0; h < 3; h++) sh.hop_out[h] = sh.hop_in[h] = 0u;
    }
    {   // the exp2 / log2 tables of the hybrid words (a pair of hybrid blocks may come)
        if (threadIdx.x < 128u) {
            const uint32_t i = threadIdx.x & 63u;
            const auto *tab = (const __attribute__((address_space(4))) uint32_t *)(threadIdx.x < 64u ? c_exp2_table : c_log2_table);
            rings[(threadIdx.x < 64u ? TAB_EXP2 : TAB_LOG2) / 4u + i] = tab[i];
        }
    }
    __syncthreads();
    if (grp * 64u >= n) return;  // (both waves of the pair: uniform)
    const uint32_t li = grp * 64u + lane;
    const bool inl = li < n && list[li] != kLaneGap;
    const uint64_t m = lmask(inl);
    if (m == 0ull) return;
    const uint32_t f = (uint32_t)__builtin_ctzll(m);
    const BlockDesc &d0 = descs[inl ? list[li] : 0u];
    const uint32_t fl = __builtin_amdgcn_readlane(d0.flags, f);
    const int32_t nt = __builtin_amdgcn_readlane(d0.num_terms, f);
    if (nt <= 5) return;  // (lane_blocks_rt's pair)
    uint8_t *rg = (uint8_t *)rings;
#define WV_RT3_ROLES(MONO_, HY_)                                                                     \
    do {                                                                                           \
        if (role == 0u) lane_parser<MONO_, HY_, LANE_RT, 16>(descs, list, n, blob, sh, rg, pair, grp, lane, dbg); \
        else if (role == 1u) lane_recon_split<MONO_, 1, RT3_NW, HY_>(descs, list, n, out, status, sh, grp, lane);  \
        else if (role == 2u) lane_recon_split<MONO_, 2, RT3_NW, HY_>(descs, list, n, out, status, sh, grp, lane);  \
        else if constexpr (RT3_NW == 3) lane_recon_split<MONO_, 3, 3, HY_>(descs, list, n, out, status, sh, grp, lane); \
    } while (0)
    if (((fl & wvf::HYBRID_FLAG) != 0) != (HYK != 0)) return;  // (the other kernel's pair)
    if (fl & wvf::MONO_DATA) WV_RT3_ROLES(true, HYK);
    else WV_RT3_ROLES(false, HYK);
#undef WV_RT3_ROLES
}

}  // namespace lane

// the term lists with a lane instantiation (decoder order, the reverse of the
// encoder's; wv_lane.hip): WavPack's fast, default and mono-default lists, and
// its 16-term 'high' lists (stereo: C3's and C5's 24-bit stereo; mono)
#define WVG_TS_FAST 17, 17
#define WVG_TS_DEFAULT -2, 3, 2, 18, 18
#define WVG_TS_M5 18, 3, 2, 18, 18
#define WVG_TS_HIGH16 2, 18, -1, 8, 6, 3, 5, 7, 4, 2, 18, -2, 3, 2, 18, 18
#define WVG_TS_MONO_HIGH16 1, 17, 2, 18, 8, 6, 3, 5, 7, 4, 2, 18, 3, 2, 18, 18
enum LaneList { LANE_FAST = 0, LANE_DEFAULT, LANE_M5, LANE_HIGH16, LANE_MONO_HIGH16, LANE_HY_DEFAULT, LANE_HY_WVC, LANE_RT };
// the lane kernel of one list over n blocks (wv_lane.hip)
// dbg (nullptr: off): per parser wave 16 words (cycles, groups by path, wait cycles: LCount)
hipError_t launch_lane(int which, dim3 grid, dim3 block, hipStream_t s, const BlockDesc *descs, const uint32_t *list,
                       uint32_t n, const uint8_t *blob, int32_t *out, uint32_t *status, uint32_t *dbg);
}  // namespace wvg
