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
// Scope: lossless PCM stereo blocks whose decorr term list is one of the
// two-wave kernel's compile-time lists, with no sticky state, wvx/wvc/exact
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
constexpr int RU = 16;                  // ring units (16 B) per lane: 16 KiB of LDS per 64-block wave
constexpr int GF = 8;                   // frames per group (refill / bound-check cadence)
constexpr int NLD = 4;                  // units a lane loads per group, at most (32 bits per word sustained)

__device__ __forceinline__ int32_t aw(int32_t w, int32_t s) {  // apply_weight (UnpackUtils.cs:703)
    return (int32_t)(((int64_t)w * (int64_t)s + 512) >> 10);
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
    // frame t (t % 8 == U): the sample-major form of decorr_stereo_pass
    // (pass_stereo, wv_decode_core.h; the ring of terms 1..8 read at t & 7, written at (t + T) & 7)
    template <int U>
    __device__ __forceinline__ void frame(int32_t &L, int32_t &R) {
        using namespace wvf;
        if constexpr (T == 17 || T == 18) {
            const int32_t sa = T == 17 ? sub32(mul32(2, hA[0]), hA[1]) : (sub32(mul32(3, hA[0]), hA[1]) >> 1);
            const int32_t oa = add32(aw(wA, sa), L);
            wA = w2::vupd(wA, sa, L, dl);
            hA[1] = hA[0];
            hA[0] = oa;
            L = oa;
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
    template <int U>
    __device__ __forceinline__ void frame(int32_t &, int32_t &) {}
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
    template <int U>
    __device__ __forceinline__ void frame(int32_t &L, int32_t &R) {
        p.template frame<U>(L, R);
        rest.template frame<U>(L, R);
    }
    __device__ __forceinline__ bool wbad() const { return p.wbad() || rest.wbad(); }
};

// Each lane's ring is RU units at rbase = lane * RSTRIDE bytes of LDS (the
// 16-B pad spreads the lanes' unit writes over the banks); dword rp (a count
// of dwords from the lane's 16-B aligned stream base) is at rbase + (rp % (4 RU)) * 4
constexpr uint32_t RSTRIDE = RU * 16u + 16u;

// bytes at or past the stream end read as 0xFF (BitsUtils.cs:125-139): unit u
// relative to a stream ending at byte e
__device__ __forceinline__ uint32_t ff_tail(uint32_t v, uint32_t pos, uint32_t e) {
    if (pos >= e) return 0xFFFFFFFFu;
    const uint32_t keep = e - pos;  // bytes of v that are real
    return keep >= 4 ? v : (v | (0xFFFFFFFFu << (keep * 8)));
}
__device__ __forceinline__ uint4 ff_unit(uint4 v, uint32_t u, uint32_t e) {
    const uint32_t b = u * 16u;
    v.x = ff_tail(v.x, b, e);
    v.y = ff_tail(v.y, b + 4, e);
    v.z = ff_tail(v.z, b + 8, e);
    v.w = ff_tail(v.w, b + 12, e);
    return v;
}

struct LState {
    uint64_t win;  // bit window, LSB = next bit; bits at or above nb are zero
    int32_t nb;    // valid bits in win (>= 33 at every word start)
    uint32_t rp;   // ring dword merged next
    uint32_t nxt;  // ring dword rp, read ahead
    uint64_t h0m, h1m;  // holding_zero / holding_one, one bit per lane (SGPR pairs)
    uint32_t zacc;
    int32_t m[2][3];
    uint32_t pmax;   // largest unary bit count of a non-held word (17: escape / bits error)
    int32_t slack;   // least window bits left after a word (< 0: a word past the window)
    uint32_t bad;
};

// c ? a : b as one v_cndmask (the compiler otherwise turns nested selects
// into divergent branches with register copies at every join)
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
    uint32_t r;
    const uint64_t m = __builtin_amdgcn_ballot_w64(c);
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ int32_t vseli(bool c, int32_t a, int32_t b) {
    return (int32_t)vsel(c, (uint32_t)a, (uint32_t)b);
}
// the same on a lane mask already in SGPRs (no compare re-derived per use)
__device__ __forceinline__ uint32_t vselm(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ int32_t vselmi(uint64_t m, int32_t a, int32_t b) {
    return (int32_t)vselm(m, (uint32_t)a, (uint32_t)b);
}
__device__ __forceinline__ uint64_t lmask(bool c) { return __builtin_amdgcn_ballot_w64(c); }
// m + 5 k (one v_lshl_add: k * 4 + k, then the add; the compiler picks a 64-bit multiply-add)
__device__ __forceinline__ int32_t add5(int32_t m, int32_t k) {
    int32_t r;
    asm("v_lshl_add_u32 %0, %1, 2, %1" : "=v"(r) : "v"(k));
    return wvf::add32(m, r);
}

// small VALU helpers the compiler does not pick on its own
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
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// window refill: keep >= 32 bits by merging the dword read ahead (then read the next)
__device__ __forceinline__ void lrefill(LState &s, const uint8_t *ring, uint32_t rbase) {
    const bool need = s.nb <= 32;
    s.win |= (uint64_t)vsel(need, s.nxt, 0u) << ((uint32_t)s.nb & 63u);
    s.nb += need ? 32 : 0;
    s.rp += need ? 1u : 0u;
    s.nxt = *(const uint32_t *)(ring + rbase + ((s.rp & (RU * 4u - 1u)) << 2));
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
template <int C>
__device__ __forceinline__ int32_t lword(LState &s, const uint8_t *ring, uint32_t rbase) {
    using namespace wvf;
    // zero-run mode (:304-352): both channels' median[0] < 2, nothing held
    const uint64_t zrm = lmask((((uint32_t)(s.m[0][0] | s.m[1][0])) & ~1u) == 0u) & ~(s.h0m | s.h1m);
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
    const uint64_t hzm = s.h0m | zm;
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
    const uint32_t ones = vselm(hzm, 0u, addc(raw >> 1, s.h1m));
    const uint64_t b0m = lmask((raw & 1u) != 0u);
    // (lanes outside this path -- the other side of a tail group's FULL/partial
    // split -- keep their bits)
    const uint64_t exm = __builtin_amdgcn_read_exec();
    s.h1m = (s.h1m & ~exm) | (~hzm & b0m);
    s.h0m = (s.h0m & ~exm) | (~hzm & ~b0m & exm);
    const int32_t m0 = s.m[C][0], m1 = s.m[C][1], m2 = s.m[C][2];
    const uint32_t a0 = (uint32_t)(m0 >> 4), a1 = (uint32_t)(m1 >> 4), a2 = (uint32_t)(m2 >> 4);
    const uint64_t o0 = lmask(ones == 0u), o1 = lmask(ones == 1u), o2 = lmask(ones == 2u), ob = o0 | o1;
    const uint32_t mc = vselm(o0, a0, vselm(o1, a1, a2));
    const uint32_t low1 = a0 + 1u;
    const uint32_t low2 = (uint32_t)mad24((int32_t)(ones > 2u ? ones - 2u : 0u), (int32_t)(a2 + 1u), (int32_t)(low1 + a1 + 1u));
    const uint32_t low = vselm(o0, 0u, vselm(o1, low1, low2));
    // median updates (:433-475; DIV0/1/2 as shifts): m + ((m + off) >> s) * mult with
    // (off, mult) = (D - 2, -2) for the bucket's own median, (D, 5) below it, (-, 0) above
    s.m[C][0] = mad24((int32_t)(add3((uint32_t)m0, 128u, (uint32_t)csel<-2, 0>(o0))) >> 7, csel<-2, 5>(o0), m0);
    s.m[C][1] = mad24((int32_t)(add3((uint32_t)m1, 64u, (uint32_t)csel<-2, 0>(o1))) >> 6,
                      vselmi(o0, 0, csel<-2, 5>(o1)), m1);
    s.m[C][2] = mad24((int32_t)(add3((uint32_t)m2, 32u, (uint32_t)csel<-2, 0>(o2))) >> 5,
                      vselmi(ob, 0, csel<-2, 5>(o2)), m2);
    // read_code(high - low = mc) (WordsUtils.cs:546-570), then the sign bit
    const uint32_t x = (uint32_t)s.win;
    const uint32_t z = (uint32_t)__builtin_clz(mc | 1u);
    const uint32_t ones_z = 0xFFFFFFFFu >> z;
    const uint32_t ex = ones_z - mc;
    const uint32_t nbt = z ^ 31u;
    const uint32_t v = x & (ones_z >> 1);
    const uint64_t bigm = lmask(v >= ex);
    const uint32_t code = vselm(bigm, 2u * v + __builtin_amdgcn_ubfe(x, nbt, 1) - ex, v);
    const uint32_t used = addc(nbt, bigm);
    const uint32_t mid = low + code;
    const int32_t sg = __builtin_amdgcn_sbfe((int32_t)x, used, 1);  // 0 or -1
    lskip(s, vselm(zm, 0u, used + 1u));
    const int32_t out = (int32_t)vselm(zm, 0u, mid ^ (uint32_t)sg);
    lrefill(s, ring, rbase);
    return out;
}

template <int... Ts>
struct LaneTerms {
    static constexpr int n = sizeof...(Ts);
    static constexpr int8_t t[sizeof...(Ts) + 1] = {(int8_t)Ts..., 0};
};

// Per-block outcome when its last frame is done (the lane keeps decoding
// garbage after it, with its stores off, so the wave's control flow stays
// uniform and the holding-flag masks stay in SGPRs)
struct LEnd {
    const BlockDesc *d;
    uint32_t *st;
    int32_t ml;
    uint32_t u0;  // units written to the ring before this group
};
__device__ __forceinline__ void lane_finish(const LState &s, const LEnd &e, int32_t mx, int32_t mn, uint32_t crc) {
    uint32_t bad = s.bad | (mx > e.ml || mn < -e.ml ? 8u : 0u) | (s.pmax >= 17u ? 16u : 0u) |
                   (s.slack < 0 ? 32u : 0u) | (s.rp >= e.u0 * 4u ? 64u : 0u);
    uint32_t st = 0;
    if (e.d->nframes == e.d->block_samples) {
        st |= ST_CRC_CHECKED;
        if ((int32_t)crc != e.d->crc) st |= ST_CRC_ERROR;
    }
    *e.st = bad ? (ST_REDO | (bad << 16)) : st;
}

// one frame t = g0 + U: two words, the passes, joint stereo, the mute bound,
// the CRC, fixup and the store.  FULL: every lane of the wave is inside its block
template <int U, bool FULL, int... Ts>
__device__ __forceinline__ void lframe(LState &s, LChain<Ts...> &ch, const uint8_t *ring, uint32_t rb, uint32_t g0,
                                       uint32_t nfr, bool joint, int32_t &mx, int32_t &mn, uint32_t &crc, uint32_t sh,
                                       int32_t *o, const LEnd &e) {
    const uint32_t t = g0 + U;
    int32_t L = lword<0>(s, ring, rb);
    int32_t R = lword<1>(s, ring, rb);
    ch.template frame<U>(L, R);
    if (joint) {
        R = wvf::sub32(R, L >> 1);
        L = wvf::add32(L, R);
    }
    mx = max(mx, max(L, R));
    mn = min(mn, min(L, R));
    // crc = (crc * 3 + L) * 3 + R (UnpackUtils.cs:620-626)
    crc = crc * 9u + (uint32_t)L * 3u + (uint32_t)R;
    int2 v;
    v.x = (int32_t)((uint32_t)L << sh);
    v.y = (int32_t)((uint32_t)R << sh);
    if (FULL) {
        *(int2 *)(o + 2u * t) = v;
    } else {
        if (t < nfr) *(int2 *)(o + 2u * t) = v;
        if (t + 1u == nfr) lane_finish(s, e, mx, mn, crc);
    }
}

template <bool FULL, int... Ts>
__device__ __forceinline__ void lgroup(LState &s, LChain<Ts...> &ch, const uint8_t *ring, uint32_t rb, uint32_t g0,
                                       uint32_t nfr, bool joint, int32_t &mx, int32_t &mn, uint32_t &crc, uint32_t sh,
                                       int32_t *o, const LEnd &e) {
    lframe<0, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<1, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<2, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<3, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<4, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<5, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<6, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
    lframe<7, FULL>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, e);
}

// can this lane decode block d exactly (else ST_REDO)?
template <int... Ts>
__device__ __forceinline__ bool lane_ok(const BlockDesc &d) {
    using namespace wvf;
    if (d.kind != KIND_PCM) return false;
    if (d.flags & (HYBRID_FLAG | MONO_DATA | FLOAT_DATA | INT32_DATA)) return false;
    if (d.inherit || d.chain_len >= 2 || d.wvx_state || d.wvc_len || d.xfloat || d.pre_end || d.fstatus) return false;
    if (d.out_off & 1u) return false;  // 8-B stores
    if (d.num_terms != (int32_t)sizeof...(Ts)) return false;
    constexpr int8_t terms[sizeof...(Ts) + 1] = {(int8_t)Ts..., 0};
    for (int i = 0; i < (int)sizeof...(Ts); i++)
        if (d.term[i] != terms[i]) return false;
    return true;
}

template <int... Ts>
__device__ __forceinline__ void lane_blocks(const BlockDesc *__restrict__ descs, const uint32_t *__restrict__ list,
                                            uint32_t n, const uint8_t *__restrict__ blob, int32_t *__restrict__ out,
                                            uint32_t *__restrict__ status) {
    using namespace wvf;
    __shared__ __attribute__((aligned(16))) uint32_t ringw[64 * RSTRIDE / 4];
    const uint8_t *ring = (const uint8_t *)ringw;
    const uint32_t lane = threadIdx.x;
    const uint32_t rb = lane * RSTRIDE;  // this lane's ring
    const uint32_t li = blockIdx.x * 64u + lane;
    // every lane stays in the wave (uniform loops keep the lane masks in SGPRs):
    // a lane past the list or with a block it does not take decodes 0 frames
    const bool inl = li < n;
    const uint32_t bi = inl ? list[li] : 0u;
    const BlockDesc &d = descs[bi];
    const bool ok = inl && lane_ok<Ts...>(d);
    if (inl && !ok) status[bi] = ST_REDO | (1u << 16);
    const uint32_t nfr = ok ? d.nframes : 0u;
    // the wave runs to its longest block; groups inside every block skip the per-frame end tests
    uint32_t nmax = nfr, nmin = nfr ? nfr : 0xFFFFFFFFu;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, off));
        nmin = min(nmin, (uint32_t)__shfl_xor((int)nmin, off));
    }
    nmax = __builtin_amdgcn_readfirstlane(nmax);
    nmin = __builtin_amdgcn_readfirstlane(nmin);
    const bool joint = (d.flags & JOINT_STEREO) != 0;
    const uint32_t sh = (uint32_t)d.shift & 31u;
    const int32_t ml = d.mute_limit;
    int32_t *o = out + d.out_off;

    // payload: 16-B units from the aligned base; bytes at or past e read 0xFF
    const uint64_t boff = d.bits_off;
    const uint4 *src = (const uint4 *)(blob + (boff & ~(uint64_t)15));
    const uint32_t skip = (uint32_t)(boff & 15u);
    const uint32_t e = ok ? skip + d.bits_len : 0u;
    const uint32_t eu = (e + 15u) >> 4;
    const uint4 ffu = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    uint8_t *ringm = (uint8_t *)ringw;
#pragma unroll 4
    for (uint32_t u = 0; u < (uint32_t)RU; u++) {
        uint4 v = u < eu ? src[u] : ffu;
        if (u + 1u >= eu) v = ff_unit(v, u, e);
        *(uint4 *)(ringm + rb + (u << 4)) = v;
    }
    uint32_t fu = RU;  // next unit to load

    LState s;
    s.rp = skip >> 2;
    s.win = (uint64_t)(*(const uint32_t *)(ring + rb + ((s.rp & (RU * 4u - 1u)) << 2))) |
            ((uint64_t)(*(const uint32_t *)(ring + rb + (((s.rp + 1u) & (RU * 4u - 1u)) << 2))) << 32);
    s.win >>= (skip & 3u) * 8u;
    s.nb = 64 - (int32_t)((skip & 3u) * 8u);
    s.rp += 2u;
    s.nxt = *(const uint32_t *)(ring + rb + ((s.rp & (RU * 4u - 1u)) << 2));
    s.h0m = s.h1m = 0ull;
    s.zacc = 0u;
    s.pmax = 0u;
    s.slack = 0;
    s.bad = 0u;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int k = 0; k < 3; k++) s.m[c][k] = d.median[c][k];
    LChain<Ts...> ch;
    ch.init(d, 0);
    uint32_t crc = 0xFFFFFFFFu;
    int32_t mx = 0, mn = 0;

    for (uint32_t g0 = 0; g0 < nmax; g0 += GF) {
        // bounds that keep the group exact (else the two-wave kernel redoes the block;
        // the reason lands in status bits 16-23 beside ST_REDO, for diagnostics)
        const int32_t mm = max(max(max(s.m[0][0], s.m[0][1]), max(s.m[0][2], s.m[1][0])), max(s.m[1][1], s.m[1][2]));
        s.bad |= (mm >= (1 << 26) ? 2u : 0u) | (ch.wbad() ? 4u : 0u);
        // this group's loads: the units after fu that fit in the ring
        const uint32_t u0 = fu;
        const uint32_t room = (s.rp >> 2) + (uint32_t)RU - u0;
        const uint32_t nld = room < (uint32_t)NLD ? room : (uint32_t)NLD;
        uint4 st0 = ffu, st1 = ffu, st2 = ffu, st3 = ffu;
        if (nld > 0u && u0 < eu) st0 = src[u0];
        if (nld > 1u && u0 + 1u < eu) st1 = src[u0 + 1u];
        if (nld > 2u && u0 + 2u < eu) st2 = src[u0 + 2u];
        if (nld > 3u && u0 + 3u < eu) st3 = src[u0 + 3u];
        fu = u0 + nld;
        const LEnd le = {&d, status + bi, ml, u0};
        if (g0 + GF < nmin)  // (strict: the group holding a block's last frame runs lane_finish)
            lgroup<true>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, le);
        else
            lgroup<false>(s, ch, ring, rb, g0, nfr, joint, mx, mn, crc, sh, o, le);
        // the reader stayed inside the units written before this group
        if (s.rp >= u0 * 4u) s.bad |= 64u;
        // the loads land in the ring (the unit holding the stream end gets its 0xFF tail)
        if (nld > 0u) {
            if (u0 + 1u >= eu) st0 = ff_unit(st0, u0, e);
            *(uint4 *)(ringm + rb + (((u0) & (RU - 1)) << 4)) = st0;
        }
        if (nld > 1u) {
            if (u0 + 2u >= eu) st1 = ff_unit(st1, u0 + 1u, e);
            *(uint4 *)(ringm + rb + (((u0 + 1u) & (RU - 1)) << 4)) = st1;
        }
        if (nld > 2u) {
            if (u0 + 3u >= eu) st2 = ff_unit(st2, u0 + 2u, e);
            *(uint4 *)(ringm + rb + (((u0 + 2u) & (RU - 1)) << 4)) = st2;
        }
        if (nld > 3u) {
            if (u0 + 4u >= eu) st3 = ff_unit(st3, u0 + 3u, e);
            *(uint4 *)(ringm + rb + (((u0 + 3u) & (RU - 1)) << 4)) = st3;
        }
    }
    // (every block with frames was finished by lane_finish in its last group)
    if (ok && nfr == 0u) status[bi] = (d.block_samples == 0u) ? ST_CRC_CHECKED | ((int32_t)0xFFFFFFFFu != d.crc ? ST_CRC_ERROR : 0u) : 0u;
}

}  // namespace lane
}  // namespace wvg
