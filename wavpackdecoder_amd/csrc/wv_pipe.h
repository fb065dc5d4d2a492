// wv_pipe.h -- the pipelined reconstruction wave: decorrelation passes of any
// term list, one pass per lane pair (lane = 2 * pass + channel; mono: lane =
// pass), frames flowing through the passes as through a systolic array.
//
// The parser wave is the one of wv_wave2.h (unchanged).  The reconstruction
// wave of wv_wave2.h runs every pass for one frame at a time with all 32 lane
// pairs computing the same values, i.e. ~12 VALU instructions per pass per
// frame and one register ring per pass: 16-term lists cost ~200 VALU per frame
// and 211 VGPRs.  Here lane pair p applies pass p (UnpackUtils.cs:688-1240) to
// frame s - p at step s, and after each step every value moves one pair up
// (DPP wave rotate), so one step advances all passes at once: ~30-40 VALU per
// frame for any list up to 16 terms, ~40 VGPRs, one kernel for every term list.
//
// Per lane: the pass's weight and history.  17/18 and terms 1, 2 read the last
// two outputs (registers s0, s1); terms 3..8 read an 8-slot ring in LDS (the
// slot for the next step is read one step ahead); stereo negative terms
// (-1/-2/-3) read the partner channel's value through a DPP quad permute, with a
// second sub-step for the channel that depends on the other's current output.
// Lanes past the last pass are identity passes (weight 0), so after step s the
// pairs D-1..31 (D = number of passes) hold the finished frames s-D+1 .. s-31.
// Every G = 33 - D steps (mono: 65 - D) one group of finished frames gets joint
// stereo, the mute test and the CRC (a power-of-9 / power-of-3 weighted wave
// sum), fixup and the store -- the same values as decode_pcm_block.  Groups
// with a mute, a bits error, or the mono crc-stop quirk take a per-frame path
// with exactly the semantics of recon_batch (wv_wave2.h).  The (short) weight
// stores at call seams (Appendix B-4) are applied per lane from a 64-bit mask of
// the seam frames of each group's window.
#pragma once
#include "wv_wave2.h"

namespace wvg {
namespace w2 {

struct PipeShared {
    Shared s;
    int32_t ring[64 * 8];  // per lane: an 8-slot history ring for terms 3..8
};

__device__ __forceinline__ int32_t wave_ror1(int32_t old, int32_t x) {
    return __builtin_amdgcn_update_dpp(old, x, 0x13C, 0xF, 0xF, false);  // wave_ror:1 (lane l <- lane l-1, 0 <- 63)
}

// sum of x over all 64 lanes (DPP row shifts + row broadcasts, then lane 63)
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int32_t)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int32_t)x, 63);
}

__device__ __forceinline__ uint32_t upow(uint32_t b, uint32_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}

// the (short)-store frames (Appendix B-4) of the caller's schedule, walked in order
struct SeamWalk {
    uint32_t cs, ce, nfr, chunk, pre_end, pre_chunk;
    bool stereo;
    __device__ __forceinline__ void init(const BlockDesc &d, bool st) {
        nfr = d.nframes;
        chunk = d.chunk;
        pre_end = d.pre_end;
        pre_chunk = d.pre_chunk;
        stereo = st;
        cs = 0;
        ce = d.first_chunk < nfr ? d.first_chunk : nfr;
    }
    __device__ __forceinline__ void next_call() {
        cs = ce;
        const uint32_t len = cs < pre_end ? min(pre_chunk, pre_end - cs) : chunk;
        ce = cs + len < nfr ? cs + len : nfr;
    }
    // bit i set when frame w0 + i (i < 64) is a seam frame; leaves the walk at
    // the first call that ends at or after w0 (windows only move forward)
    __device__ __forceinline__ uint64_t mask(int64_t w0) {
        while (cs < nfr && (int64_t)ce <= w0) next_call();
        uint64_t m = 0;
        uint32_t c0 = cs, c1 = ce;
        for (int guard = 0; guard < 130 && c0 < nfr && (int64_t)c0 < w0 + 64; guard++) {
            const int64_t e = (int64_t)c1 - 1 - w0;
            if (e >= 0 && e < 64) m |= 1ull << e;
            if (stereo && c1 - c0 >= 16) {
                const int64_t e8 = (int64_t)c0 + 7 - w0;
                if (e8 >= 0 && e8 < 64) m |= 1ull << e8;
            }
            c0 = c1;
            const uint32_t len = c0 < pre_end ? min(pre_chunk, pre_end - c0) : chunk;
            c1 = c0 + len < nfr ? c0 + len : nfr;
        }
        return m;
    }
};

// per-lane pass state and constants
struct PipeLane {
    int32_t w, s0, s1, h, pr;
    int32_t delta, lo, hi;
    uint32_t waddr, raddr;  // LDS byte addresses of this step's ring write / next step's ring read
    bool c17, c18, c1, c2, cring, cneg, second, hupd;
};

// Frames of one group through joint stereo, mute, CRC, fixup and the store, one
// at a time, exactly as recon_batch (non-lean) does: the path for groups with a
// mute, a bits error or the mono crc-stop quirk.  Values come from `v` (this
// step's outputs): frame t lives in lane pair q = s - t (mono: lane q).
// Returns the frame that muted (or -1).
template <int LAYOUT>
__device__ __forceinline__ int group_slow(int32_t v, uint32_t s, uint32_t g0, uint32_t g1, uint32_t tvalid, bool joint,
                                          const Fixup &fx, int32_t ml, int32_t &crc, Seams &sm, int32_t *out,
                                          uint64_t skip, int lane) {
    using namespace wvf;
    constexpr bool MONO = LAYOUT != 0;
    constexpr int OCH = LAYOUT == 1 ? 1 : 2;
    for (uint32_t t = g0; t <= g1; t++) {
        if (t >= tvalid) return -2;  // bits error: the caller mutes the chunk
        const uint32_t q = s - t;
        int32_t L, R = 0;
        if (MONO) {
            L = __builtin_amdgcn_readlane(v, (int)q);
            if (!sm.crc_stop && iabs(L) > ml) {
                const uint32_t qq = sm.bsp + (t - sm.chunk_start);  // absolute buffer index (B-6)
                if (qq != sm.chunk_end - sm.chunk_start) return (int)t;
                sm.crc_stop = true;
            }
            if (!sm.crc_stop) crc = add32(mul32(crc, 3), L);
        } else {
            L = __builtin_amdgcn_readlane(v, (int)(2 * q));
            R = __builtin_amdgcn_readlane(v, (int)(2 * q + 1));
            if (joint) {
                R = sub32(R, L >> 1);
                L = add32(L, R);
            }
            if (iabs(L) > ml || iabs(R) > ml) return (int)t;
            crc = add32(mul32(crc, 9), add32(mul32(L, 3), R));
        }
        const uint64_t o = (uint64_t)t * OCH;
        if (LAYOUT == 0) {
            if (lane == 0 && o >= skip) out[o] = fixup_tail(fx, L);
            if (lane == 1 && o + 1 >= skip) out[o + 1] = fixup_tail(fx, R);
        } else if (LAYOUT == 1) {
            if (lane == 0 && o >= skip) out[o] = fixup_tail(fx, L);
        } else {
            const int32_t f = fixup_tail(fx, L);
            if (lane < 2 && o + lane >= skip) out[o + lane] = f;
        }
        if (t == sm.chunk_end - 1) {
            sm.chunk_start = t + 1;
            const uint32_t len = sm.chunk_start < sm.pre_end ? min(sm.pre_chunk, sm.pre_end - sm.chunk_start) : sm.chunk;
            sm.chunk_end = sm.chunk_start + len < sm.nfr ? sm.chunk_start + len : sm.nfr;
            sm.seam8 = (!MONO && sm.chunk_end - sm.chunk_start >= 16) ? sm.chunk_start + 7 : 0xFFFFFFFFu;
            sm.bsp = 0;
            sm.crc_stop = false;
        }
    }
    return -1;
}

// chunk bookkeeping across frames [.., t1] that the fast path handled
__device__ __forceinline__ void seams_to(Seams &sm, uint32_t t1, bool mono) {
    while (sm.chunk_end - 1 <= t1 && sm.chunk_start < sm.nfr) {
        sm.chunk_start = sm.chunk_end;
        const uint32_t len = sm.chunk_start < sm.pre_end ? min(sm.pre_chunk, sm.pre_end - sm.chunk_start) : sm.chunk;
        sm.chunk_end = sm.chunk_start + len < sm.nfr ? sm.chunk_start + len : sm.nfr;
        sm.seam8 = (!mono && sm.chunk_end - sm.chunk_start >= 16) ? sm.chunk_start + 7 : 0xFFFFFFFFu;
        sm.bsp = 0;
        sm.crc_stop = false;
        if (sm.chunk_start >= sm.nfr) break;
    }
}

// one step: every lane applies its pass to its frame; returns the outputs
template <bool NEG12, bool TRUNC, bool FILL>
__device__ __forceinline__ int32_t pipe_step(PipeLane &p, int32_t x, const int32_t *ring_lds, int32_t *ring_w,
                                             uint32_t s, int q, uint64_t tmask, int64_t w0) {
    using namespace wvf;
    const bool act = !FILL || (uint32_t)q <= s;
    // prediction by class (UnpackUtils.cs:701-918; 17: 2s1-s2, 18: (3s1-s2)>>1, 1..8: s_t-term)
    const int32_t a17 = sub32(add32(p.s0, p.s0), p.s1);
    const int32_t a18 = add32(a17, p.s0) >> 1;
    int32_t pred = p.c18 ? a18 : a17;
    pred = p.c1 ? p.s0 : pred;
    pred = p.c2 ? p.s1 : pred;
    pred = p.cring ? p.pr : pred;
    pred = p.cneg ? p.h : pred;
    int32_t o = add32(x, apply_weight(p.w, pred));
    int32_t wn = vupd(p.w, pred, x, p.delta);
    if (NEG12) {  // -1: B from A's output of this frame; -2: A from B's
        const int32_t y = swap_pair(o);
        const int32_t o2 = add32(x, apply_weight(p.w, y));
        const int32_t w2 = vupd(p.w, y, x, p.delta);
        o = p.second ? o2 : o;
        wn = p.second ? w2 : wn;
    }
    wn = max(p.lo, min(p.hi, wn));
    if (TRUNC) {  // (short) store after this lane's frame when it is a seam frame (B-4)
        const int64_t bit = (int64_t)s - q - w0;
        const bool seam = bit >= 0 && bit < 64 && ((tmask >> (uint64_t)(bit & 63)) & 1ull);
        wn = seam ? (int32_t)(int16_t)wn : wn;
    }
    const int32_t hs = swap_pair(o);
    if (act) {
        p.w = wn;
        p.h = p.hupd ? hs : p.h;
        p.s1 = p.s0;
        p.s0 = o;
        *(int32_t *)((char *)ring_w + p.waddr) = o;
    }
    p.pr = *(const int32_t *)((const char *)ring_lds + p.raddr);
    p.waddr = (p.waddr & ~31u) | ((p.waddr + 4u) & 31u);
    p.raddr = (p.raddr & ~31u) | ((p.raddr + 4u) & 31u);
    return o;
}

template <int LAYOUT, bool NEG12>
__device__ __forceinline__ void recon_pipe(const BlockDesc &d, PipeShared &ps, int32_t *out_base, uint32_t *status_out,
                                           uint32_t *exc_out, int lane) {
    using namespace wvf;
    constexpr bool MONO = LAYOUT != 0;
    constexpr int WPF = MONO ? 1 : 2;      // residual words per frame
    constexpr int OCH = LAYOUT == 1 ? 1 : 2;
    constexpr int P = MONO ? 64 : 32;      // passes the wave holds
    Shared &sh = ps.s;
    const uint32_t flags = d.flags;
    const bool joint = (flags & JOINT_STEREO) != 0;
    const int32_t ml = d.mute_limit;
    const uint32_t nfr = d.nframes;
    int32_t *out = out_base + d.out_off;
    const uint64_t skip = (uint64_t)d.pre_end * OCH;
    const int nt = d.num_terms;
    const int D = nt > 0 ? nt : 1;
    const uint32_t G = (uint32_t)(P - D + 1);
    const int q = MONO ? lane : (lane >> 1);
    const bool isB = !MONO && (lane & 1);

    // ---- lane state: pass q of this lane's channel (identity past the last pass)
    PipeLane p;
    int T = q < nt ? (int)d.term[q] : 1;
    if (MONO && !(T == 17 || T == 18 || (T >= 1 && T <= 8))) T = (T & 7) == 0 ? 8 : (T & 7);  // B-12
    const int32_t *sam = q < nt ? (isB ? d.samples_B[q] : d.samples_A[q]) : nullptr;
    p.w = q < nt ? (isB ? d.weight_B[q] : d.weight_A[q]) : 0;
    p.delta = q < nt ? (int32_t)d.delta[q] : 0;
    p.c17 = T == 17;
    p.c18 = T == 18;
    p.c1 = T == 1;
    p.c2 = T == 2;
    p.cring = T >= 3 && T <= 8;
    p.cneg = T < 0;
    p.second = (T == -1 && isB) || (T == -2 && !isB);
    p.hupd = T == -3 || (T == -1 && !isB) || (T == -2 && isB);
    p.lo = p.cneg ? -1024 : INT32_MIN;
    p.hi = p.cneg ? 1024 : INT32_MAX;
    p.s0 = p.s1 = p.h = p.pr = 0;
    int32_t *ring = ps.ring;
    const uint32_t rbase = (uint32_t)lane * 32u;
    for (int i = 0; i < 8; i++) ring[lane * 8 + i] = 0;
    if (sam) {
        if (T >= 17) {
            p.s0 = sam[0];
            p.s1 = sam[1];
        } else if (T >= 1) {
            // samples[i] = output (i - T): the ring slot of frame f is f & 7
            for (int i = 0; i < 8; i++)
                if (i < T) ring[lane * 8 + ((i - T) & 7)] = sam[i];
            p.s0 = sam[T - 1];
            p.s1 = T >= 2 ? sam[T - 2] : 0;
        } else {
            p.h = sam[0];
        }
    }
    // frame t = s - q: ring write slot t & 7, read slot for the next frame (t + 1 - T) & 7
    const int Tr = p.cring ? T : 3;
    p.waddr = rbase + (uint32_t)((-q) & 7) * 4u;
    p.raddr = rbase + (uint32_t)((1 - q - Tr) & 7) * 4u;
    __builtin_amdgcn_wave_barrier();
    p.pr = *(const int32_t *)((const char *)ring + rbase + (uint32_t)((0 - q - Tr) & 7) * 4u);
    // per-lane CRC weights of a full group: frame of pair qq = s - qq, the group's last
    // frame is in pair D-1, so the weight is 9^(qq-(D-1)) (mono: 3^(qq-(D-1)))
    const uint32_t gbase = MONO ? 3u : 9u;
    const bool in_group = q >= D - 1 && (MONO || !isB);
    const uint32_t cw = in_group ? upow(gbase, (uint32_t)(q - (D - 1))) : 0u;
    const uint32_t gpow = upow(gbase, G);

    Fixup fx;
    fixup_init(fx, d);
    uint32_t status = 0;
    int32_t crc = -1;
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
    SeamWalk sw;
    sw.init(d, !MONO);

    // residual injection: lanes P*WPF-WPF.. take frame s+1's words before the rotate
    const bool inj = MONO ? lane == 63 : lane >= 62;
    const int wsel = MONO ? 0 : (lane & 1);
    uint32_t produced = 0, tvalid = nfr;
    bool stopped = false;
    // first frame's residuals into pair 0
    int32_t x = 0;

    // step blocks of G steps; the last one finishes frame nfr-1 (at step nfr + D - 2)
    const uint32_t send = nfr + (uint32_t)D - 2;
    for (uint32_t s = 0; nfr > 0 && s <= send && !stopped; s += G) {
        // residuals for frames up to s + G (the step block reads one frame ahead)
        const uint32_t fneed = min(s + G + 1, nfr);
        const uint32_t need = fneed * WPF;
        uint32_t spins = 0, perr = 0;
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
        if (perr == DEC_EXCEPTION || perr == DEC_TIMEOUT) {
            status |= perr == DEC_EXCEPTION ? ST_EXCEPTION : ST_TIMEOUT;
            if (lane == 0) *exc_out = produced / WPF;
            lds_store_rel(&sh.stop, 1);
            break;
        }
        if (perr) tvalid = min(tvalid, produced / WPF);  // bits error: frames from here are invalid
        if (s == 0) {
            const int32_t r0 = sh.res[(uint32_t)wsel % RES_RING];
            x = (q == 0) ? r0 : 0;
        }
        // the seam frames any pass touches in this step block: [s - D + 1, s + G - 1]
        const int64_t w0 = (int64_t)s - D + 1;
        const uint64_t tm = sw.mask(w0);
        const uint32_t s1 = s + G;
        int32_t v = 0;
        for (uint32_t ss = s; ss < s1; ss++) {
            // the next frame's residual words, read now, injected after the step
            const int32_t rn = sh.res[(uint32_t)((ss + 1) * WPF + wsel) % RES_RING];
            if (ss < (uint32_t)D - 1) {
                v = tm ? pipe_step<NEG12, true, true>(p, x, ring, ring, ss, q, tm, w0)
                       : pipe_step<NEG12, false, true>(p, x, ring, ring, ss, q, tm, w0);
            } else if (tm) {
                v = pipe_step<NEG12, true, false>(p, x, ring, ring, ss, q, tm, w0);
            } else {
                v = pipe_step<NEG12, false, false>(p, x, ring, ring, ss, q, tm, w0);
            }
            int32_t z = inj ? rn : v;
            x = wave_ror1(z, z);
            if (!MONO) x = wave_ror1(x, x);
        }
        // release the residual words of the frames injected so far
        lds_publish(&sh.consumed, min(s1 + 1, nfr) * WPF);
        // ---- the group of frames finished after step s1 - 1: [s1 - 1 - (P - 1), s1 - 1 - (D - 1)]
        const uint32_t sl = s1 - 1;
        const int64_t g0s = (int64_t)sl - (P - 1);
        const uint32_t g0 = g0s < 0 ? 0u : (uint32_t)g0s;
        const int64_t g1s = (int64_t)sl - (D - 1);
        if (g1s < 0) continue;
        const uint32_t g1 = min((uint32_t)g1s, nfr - 1);
        if (g0 > g1) continue;
        // values of this lane's frame after joint stereo
        const int64_t tl64 = (int64_t)sl - q;
        const uint32_t tl = (uint32_t)tl64;
        const bool valid = q >= D - 1 && tl64 >= (int64_t)g0 && tl64 <= (int64_t)g1 && tl < tvalid;
        int32_t L = v, R = 0;
        if (!MONO) {
            const int32_t y = swap_pair(v);
            L = isB ? y : v;
            R = isB ? v : y;
            if (joint) {
                R = sub32(R, L >> 1);
                L = add32(L, R);
            }
        }
        const bool bad = valid && (iabs(L) > ml || (!MONO && iabs(R) > ml));
        const bool fast = g1 < tvalid && !any_lane(bad) && !(MONO && sm.crc_stop);
        if (fast) {
            // CRC over the group: crc * base^n + sum base^(g1 - t) * v_t
            const uint32_t n = g1 - g0 + 1;
            const uint32_t vt = MONO ? (uint32_t)L : (uint32_t)add32(mul32(L, 3), R);
            // weights are for a group ending in pair D-1; a short last group ends
            // in a higher pair: divide by base^(missing) via the odd inverse
            const uint32_t sh_extra = (uint32_t)((int64_t)sl - (D - 1) - g1);  // frames past g1 in pairs < q(g1)
            uint32_t wgt = valid ? cw : 0u;
            const uint32_t sum = wave_sum(vt * wgt);
            // cw = base^(q - (D-1)) = base^(g1 - t + sh_extra): remove base^sh_extra
            // with the inverse of the (odd) base mod 2^32
            const uint32_t adj = sh_extra ? sum * upow(MONO ? 0xAAAAAAABu : 0x38E38E39u, sh_extra) : sum;
            const uint32_t pw = n == G ? gpow : upow(gbase, n);
            crc = (int32_t)((uint32_t)crc * pw + adj);
            // fixup + store (each lane its own value; mono layouts lane q -> frame tl)
            if (valid) {
                if (LAYOUT == 0) {
                    const int32_t fl = fixup_tail(fx, isB ? R : L);
                    const uint64_t o = (uint64_t)tl * 2 + (isB ? 1 : 0);
                    if (o >= skip) out[o] = fl;
                } else if (LAYOUT == 1) {
                    const uint64_t o = (uint64_t)tl;
                    if (o >= skip) out[o] = fixup_tail(fx, L);
                } else {
                    const int32_t fl = fixup_tail(fx, L);
                    const uint64_t o = (uint64_t)tl * 2;
                    if (o >= skip) out[o] = fl;
                    if (o + 1 >= skip) out[o + 1] = fl;
                }
            }
            seams_to(sm, g1, MONO);
            continue;
        }
        // per-frame path (mute, bits error, crc-stop quirk)
        const int m = group_slow<LAYOUT>(v, sl, g0, g1, tvalid, joint, fx, ml, crc, sm, out, skip, lane);
        if (m != -1) {
            if (m == -2) {
                status |= ST_BITS_ERROR;
                crc_garbage = true;
                if (MONO && sm.chunk_start == 0 && sm.bsp > 0) status |= ST_NONDET;
            }
            status |= ST_MUTED;
            lds_store_rel(&sh.stop, 1);
            const int32_t z0 = fixup_tail(fx, 0);
            mute_fill<OCH>(sm.chunk_end, nfr, z0, z0, out, sm.chunk_start, skip, lane);
            stopped = true;
        }
    }
    if (!(status & (ST_EXCEPTION | ST_TIMEOUT)) && nfr == d.block_samples) {
        status |= ST_CRC_CHECKED;
        if (crc_garbage || crc != d.crc) status |= ST_CRC_ERROR;
    }
    if (lane == 0) *status_out = d.fstatus | status;
}

template <bool NEG12>
__device__ __forceinline__ void block_pipe(const BlockDesc *descs, const uint32_t *list, const uint8_t *blob,
                                           int32_t *out, uint32_t *status, uint32_t *aux) {
    __shared__ PipeShared ps;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t bi = list[blockIdx.x];
    const BlockDesc &d = descs[bi];
    if (threadIdx.x == 0) {
        ps.s.produced = 0;
        ps.s.consumed = 0;
        ps.s.err = 0;
        ps.s.stop = 0;
        ps.s.pos = 0;
    }
    __syncthreads();
    if (wave == 0) {
        parser(d, blob, ps.s, lane);
    } else {
        const uint32_t f = d.flags;
        if (f & wvf::FALSE_STEREO)
            recon_pipe<2, false>(d, ps, out, &status[bi], &aux[bi], lane);
        else if (f & wvf::MONO_FLAG)
            recon_pipe<1, false>(d, ps, out, &status[bi], &aux[bi], lane);
        else
            recon_pipe<0, NEG12>(d, ps, out, &status[bi], &aux[bi], lane);
    }
}

}  // namespace w2
}  // namespace wvg
