// wv_decode_core.h -- per-block WavPack PCM decode, sample-major.
//
// This is the reference's hot path (WavPackUtils.WavpackUnpackSamples ->
// UnpackUtils.unpack_samples, WavPackUtils.cs:200-282 / UnpackUtils.cs:510-686)
// re-expressed for one block at a time and one frame at a time:
//
//   get_words           WordsUtils.cs:272-511  (entropy decode of the residuals)
//   decorr passes       UnpackUtils.cs:688-1240 (adaptive prediction, every pass)
//   joint stereo + CRC + mute          UnpackUtils.cs:549-664
//   fixup_samples / float_values       UnpackUtils.cs:1251-1404, FloatUtils.cs:32-56
//   FALSE_STEREO duplication           UnpackUtils.cs:668-680
//   check_crc_error                    UnpackUtils.cs:1414-1421
//
// The reference evaluates pass-major over each caller chunk (4096 frames in
// WvDemo).  Sample-major gives the same values except at three chunk seams,
// which are emulated from the descriptor's chunk schedule:
//   * weights are stored back as (short) at the end of every pass call and
//     after the first 8 frames of stereo chunks >= 16 frames (Appendix B-4);
//   * muting zeroes the whole chunk and every later chunk (Appendix B-5);
//   * the mono mute test compares an absolute buffer index (Appendix B-6).
//
// The code is __host__ __device__: the HIP kernel (wv_decode.hip) runs it one
// block per lane, and tests/emu builds it for the host so the logic can be
// checked against the oracle on a machine without a GPU.
#pragma once
#include <stdint.h>

#include "wv_desc.h"
#include "wv_format.h"

namespace wvg {

#if defined(__HIPCC__)
__constant__ __attribute__((aligned(16))) uint8_t c_exp2_table[256] = {WVF_EXP2_TABLE};
__constant__ __attribute__((aligned(16))) uint8_t c_log2_table[256] = {WVF_LOG2_TABLE};
// A byte table read as the dword holding the byte, through the constant address
// space: with a wave-uniform index (the parser wave, the wave-per-block kernels)
// that is a scalar-cache load instead of a vector byte load and its memory
// latency on the serial path; a divergent index still compiles to a vector load.
__device__ __forceinline__ int tab_byte(const uint8_t *t, int i) {
    typedef const __attribute__((address_space(4))) uint32_t *cdw;
    return (int)((((cdw)t)[(unsigned)i >> 2] >> (((unsigned)i & 3u) * 8u)) & 0xFFu);
}
#endif

WVF_HD int tab_exp2(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return tab_byte(c_exp2_table, i);
#else
    return wvf::host_exp2_table[i];
#endif
}
WVF_HD int tab_log2(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return tab_byte(c_log2_table, i);
#else
    return wvf::host_log2_table[i];
#endif
}

enum { DEC_OK = 0, DEC_BITS_ERROR = 1, DEC_EXCEPTION = 2, DEC_TIMEOUT = 3 };

// the exp2 / log2 byte tables through memory (scalar cache on the device)
struct MemTabs {
    WVF_HD int exp2(int i) const { return tab_exp2(i); }
    WVF_HD int log2(int i) const { return tab_log2(i); }
};

// exp2s (WordsUtils.cs:633-646); int.MinValue recurses forever in C# -> exception
template <class TB = MemTabs>
WVF_HD int32_t dev_exp2s(int32_t log, int &exc, const TB &tb = TB()) {
    bool neg = log < 0;
    if (log == INT32_MIN) {
        exc = 1;
        return 0;
    }
    if (neg) log = -log;
    int64_t value = tb.exp2(log & 0xff) | 0x100;
    int e = log >> 8;
    int32_t r = (e <= 9) ? (int32_t)wvf::sar64(value, 9 - e) : (int32_t)wvf::shl64(value, e - 9);
    return neg ? (int32_t)(0u - (uint32_t)r) : r;
}

// mylog2 (WordsUtils.cs:588-608); out-of-table indices are C# exceptions
template <class TB = MemTabs>
WVF_HD int dev_mylog2(int64_t avalue, int &exc, const TB &tb = TB()) {
    avalue += avalue >> 9;
    if (avalue < 0 || avalue >= (1LL << 32)) {
        exc = 1;
        return 0;
    }
    uint32_t a = (uint32_t)avalue;
    int dbits = a ? 32 - __builtin_clz(a) : 0;
    if (a < 256) return (dbits << 8) + tb.log2((int)(((uint64_t)a << (9 - dbits)) & 0xff));
    return (dbits << 8) + tb.log2((int)((a >> (dbits - 9)) & 0xff));
}

// ---------------------------------------------------------------------------
// Bit reader over the batch blob: the byte-serial LSB-first Bitstream of
// BitsUtils.cs:15-68 as a 64-bit window.  Bytes at or past `end` read as
// 0xFF (bs_read fills the buffer with -1 once ptr reaches end, :125-139).
// ---------------------------------------------------------------------------
struct BitReader {
    const uint8_t *base;
    uint64_t pos, end, start;
    uint64_t win;
    int nb;

    WVF_HD void init(const uint8_t *blob, uint64_t off, uint64_t len) {
        base = blob;
        pos = start = off;
        end = off + len;
        win = 0;
        nb = 0;
    }
    // bits consumed since the (byte-aligned) start
    WVF_HD uint64_t consumed() const { return (pos - start) * 8 - (uint64_t)nb; }
    // keep at least 33 valid bits in the window
    WVF_HD void refill() {
#if defined(__HIP_DEVICE_COMPILE__)
        // the device: the 8 bytes from pos out of three aligned dwords read together
        // through the scalar cache (a decode here is wave-uniform) instead of one
        // dependent byte load per byte; the byte loop only within 12 bytes of the end
        if (nb <= 56 && pos + 12u <= end) {
            typedef const __attribute__((address_space(4))) uint32_t *cdw;
            const cdw w = (cdw)(base + (pos & ~(uint64_t)3));  // (base: the blob, 16-B aligned)
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
            const uint32_t sh = (uint32_t)(pos & 3u) * 8u;
            uint64_t v = ((uint64_t)w1 << 32) | w0;
            if (sh) v = (v >> sh) | ((uint64_t)w2 << (64u - sh));
            const int k = (64 - nb) >> 3;  // bytes taken: nb ends in 57..64, as the byte loop's
            win |= (k >= 8 ? v : (v & ((1ull << (8 * k)) - 1ull))) << nb;
            nb += 8 * k;
            pos += (uint64_t)k;
            return;
        }
#endif
        while (nb <= 56) {
            uint64_t b = pos < end ? (uint64_t)base[pos] : 0xFFull;
            win |= b << nb;
            nb += 8;
            pos++;
        }
    }
    WVF_HD void need(int n) {
        if (nb < n) refill();
    }
    WVF_HD void skip(int n) {
        win >>= n;
        nb -= n;
    }
    WVF_HD int getbit() {
        need(1);
        int b = (int)(win & 1);
        skip(1);
        return b;
    }
    // n <= 32 (masked result, as every reference caller masks)
    WVF_HD uint32_t getbits(int n) {
        if (n <= 0) return 0;
        need(n);
        uint32_t v = (uint32_t)(win & ((n == 64) ? ~0ull : ((1ull << n) - 1)));
        skip(n);
        return v;
    }
    // BitsUtils.getbits (:37-68) as its callers see it: the returned value is
    // the unmasked shift register, i.e. every bit up to the byte boundary the
    // read stops at (at most 32), not just the n bits consumed.  n <= 32.
    WVF_HD uint32_t getbits_reg(int n) {
        const uint64_t p = consumed();
        int bc = n + (int)((8u - ((uint32_t)(p + (uint64_t)n) & 7u)) & 7u);
        if (bc > 32) bc = 32;
        need(bc);
        uint32_t v = (uint32_t)(win & ((1ull << bc) - 1));
        skip(n);
        return v;
    }
    // BitsUtils.getbits for n > 32 (INT32 sent_bits of a malformed ID_INT32_INFO, up to
    // 255): the reference loads bytes into its 32-bit register at shift bc & 31 until bc
    // reaches n -- bytes past 32 bits wrap onto the low ones (C#'s masked int shift) --
    // and returns the register; afterwards its state is that of n bits consumed.
    WVF_HD uint32_t getbits_big(int n) {
        const uint64_t p = consumed();
        uint32_t bc = (8u - (uint32_t)(p & 7u)) & 7u;  // bits left of the byte in the register
        uint64_t nb8 = (p + 7u) >> 3;                 // the next byte the reference loads
        auto byte_at = [&](uint64_t i) -> uint32_t { return start + i < end ? base[start + i] : 0xFFu; };
        uint32_t sr = bc ? byte_at(nb8 - 1u) >> (8u - bc) : 0u;
        while ((int)bc < n) {
            sr |= byte_at(nb8) << (bc & 31u);
            bc += 8u;
            nb8++;
        }
        int left = n;
        while (left > 32) {
            need(32);
            skip(32);
            left -= 32;
        }
        need(left);
        skip(left);
        return sr;
    }
    // consume a run of one bits the way the reference's getbit loops do
    // (WordsUtils.cs:321, 381, 391): up to `cap` ones, plus the terminating
    // zero when fewer than `cap` were found.  cap <= 40.
    WVF_HD int consume_ones(int cap) {
        need(cap + 1);
        uint64_t inv = ~win;
        int r = inv ? __builtin_ctzll(inv) : 64;
        if (r >= cap) {
            skip(cap);
            return cap;
        }
        skip(r + 1);
        return r;
    }
};

// ---------------------------------------------------------------------------
// entropy state: words_data + entropy_data (words_data.cs, entropy_data.cs)
// ---------------------------------------------------------------------------
struct Entropy {
    int32_t med[2][3];
    int32_t slow[2];
    int32_t errlim[2];
    int64_t acc[2], dlt[2];
    int64_t zeros_acc;
    int32_t h1, h0;  // holding_one / holding_zero as 0/1 (ints keep them in SGPRs on the GPU)
};

// update_error_limit (WordsUtils.cs:195-261)
template <class TB = MemTabs>
WVF_HD void update_error_limit(Entropy &w, uint32_t flags, int &exc, const TB &tb = TB()) {
    using namespace wvf;
    int32_t bitrate_0 = (int32_t)((w.acc[0] += w.dlt[0]) >> 16);
    if (flags & MONO_DATA) {
        if (flags & HYBRID_BITRATE) {
            int32_t slow_log_0 = add32(w.slow[0], SLO) >> SLS;
            w.errlim[0] = (sub32(slow_log_0, bitrate_0) > -0x100) ? dev_exp2s(add32(sub32(slow_log_0, bitrate_0), 0x100), exc, tb) : 0;
        } else
            w.errlim[0] = dev_exp2s(bitrate_0, exc, tb);
    } else {
        int32_t bitrate_1 = (int32_t)((w.acc[1] += w.dlt[1]) >> 16);
        if (flags & HYBRID_BITRATE) {
            int32_t slow_log_0 = add32(w.slow[0], SLO) >> SLS;
            int32_t slow_log_1 = add32(w.slow[1], SLO) >> SLS;
            if (flags & HYBRID_BALANCE) {
                int32_t balance = add32(add32(sub32(slow_log_1, slow_log_0), bitrate_1), 1) >> 1;
                if (balance > bitrate_0) {
                    bitrate_1 = mul32(bitrate_0, 2);
                    bitrate_0 = 0;
                } else if ((int32_t)(0u - (uint32_t)balance) > bitrate_0) {
                    bitrate_0 = mul32(bitrate_0, 2);
                    bitrate_1 = 0;
                } else {
                    bitrate_1 = add32(bitrate_0, balance);
                    bitrate_0 = sub32(bitrate_0, balance);
                }
            }
            w.errlim[0] = (sub32(slow_log_0, bitrate_0) > -0x100) ? dev_exp2s(add32(sub32(slow_log_0, bitrate_0), 0x100), exc, tb) : 0;
            w.errlim[1] = (sub32(slow_log_1, bitrate_1) > -0x100) ? dev_exp2s(add32(sub32(slow_log_1, bitrate_1), 0x100), exc, tb) : 0;
        } else {
            w.errlim[0] = dev_exp2s(bitrate_0, exc, tb);
            w.errlim[1] = dev_exp2s(bitrate_1, exc, tb);
        }
    }
}

// read_code (WordsUtils.cs:546-570) with count_bits (:513-537); false: the
// nbits_table[] index is out of range (the C# throws)
template <class BR>
WVF_HD bool read_code(BR &bs, int64_t maxcode, int64_t &code) {
    if (maxcode < 0 || maxcode >= (1LL << 32)) return false;
    const uint32_t mc = (uint32_t)maxcode;
    const int bitcount = mc ? 32 - __builtin_clz(mc) : 0;
    code = 0;
    if (bitcount != 0) {
        const int64_t extras = (int64_t)wvf::shl32(1, bitcount) - maxcode - 1;
        code = (int64_t)(bs.getbits(bitcount - 1) & (uint32_t)(wvf::shl32(1, bitcount - 1) - 1));
        if (code >= extras) {
            code = (code << 1) - extras;
            if (bs.getbit()) ++code;
        }
    }
    return true;
}

// One residual of get_words (WordsUtils.cs:290-503).  `c` is entidx, `even`
// is ((csamples & 1) == 0).  Returns DEC_* and the value in `out`.
// With a .wvc correction stream `cb` (beyond the reference, which never reads
// it; WavPack 4's get_word): a word the error limit left inexact reads its exact
// magnitude as read_code(wvcbits, high - low) + low, and *corr receives the
// exact residual minus the lossy one (0 for every other word).
template <class BR, class TB = MemTabs>
WVF_HD int get_word(Entropy &w, BR &bs, uint32_t flags, int c, bool even, int32_t &out, const TB &tb = TB(),
                    BR *cb = nullptr, int32_t *corr = nullptr) {
    using namespace wvf;
    int exc = 0;
    if (corr) *corr = 0;
    const bool mono = (flags & MONO_DATA) != 0;
    if ((w.med[0][0] & ~1) == 0 && !w.h0 && !w.h1 && (w.med[1][0] & ~1) == 0) {
        // zero-run mode (:304-352)
        if (w.zeros_acc > 0) {
            if (--w.zeros_acc > 0) {
                w.slow[c] = sub32(w.slow[c], add32(w.slow[c], SLO) >> SLS);
                out = 0;
                return DEC_OK;
            }
        } else {
            int cbits = bs.consume_ones(33);
            if (cbits == 33) return DEC_BITS_ERROR;
            if (cbits < 2)
                w.zeros_acc = cbits;
            else
                w.zeros_acc = (int64_t)bs.getbits(cbits - 1) | ((int64_t)1 << (cbits - 1));
            if (w.zeros_acc > 0) {
                w.slow[c] = sub32(w.slow[c], add32(w.slow[c], SLO) >> SLS);
                for (int k = 0; k < 3; k++) w.med[0][k] = w.med[1][k] = 0;
                out = 0;
                return DEC_OK;
            }
        }
    }

    int32_t ones;
    if (w.h0) {
        w.h0 = false;
        ones = 0;
    } else {
        // unary count with LIMIT_ONES escape (:361-409): leading ones, capped at 17
        int u = bs.consume_ones(17);
        if (u == 17) return DEC_BITS_ERROR;
        ones = u;
        if (u == LIMIT_ONES) {
            int cbits = bs.consume_ones(33);
            if (cbits == 33) return DEC_BITS_ERROR;
            if (cbits < 2)
                ones = cbits;
            else
                ones = (int32_t)(bs.getbits(cbits - 1) | (uint32_t)shl32(1, cbits - 1));
            ones = add32(ones, LIMIT_ONES);
        }
        if (w.h1) {
            w.h1 = (ones & 1) != 0;
            ones = add32(ones >> 1, 1);
        } else {
            w.h1 = (ones & 1) != 0;
            ones >>= 1;
        }
        w.h0 = !w.h1;
    }

    if ((flags & HYBRID_FLAG) && (mono || even)) update_error_limit(w, flags, exc, tb);

    int32_t *m = w.med[c];
    int64_t low, high;
    if (ones == 0) {
        low = 0;
        high = (int64_t)add32(m[0] >> 4, 1) - 1;
        m[0] = sub32(m[0], mul32(add32(m[0], 126) >> 7, 2));
    } else {
        low = add32(m[0] >> 4, 1);
        m[0] = add32(m[0], mul32(add32(m[0], 128) >> 7, 5));
        if (ones == 1) {
            high = low + add32(m[1] >> 4, 1) - 1;
            m[1] = sub32(m[1], mul32(add32(m[1], 62) >> 6, 2));
        } else {
            low += add32(m[1] >> 4, 1);
            m[1] = add32(m[1], mul32(add32(m[1], 64) >> 6, 5));
            if (ones == 2) {
                high = low + add32(m[2] >> 4, 1) - 1;
                m[2] = sub32(m[2], mul32(add32(m[2], 30) >> 5, 2));
            } else {
                low += (int64_t)mul32(sub32(ones, 2), add32(m[2] >> 4, 1));
                high = low + add32(m[2] >> 4, 1) - 1;
                m[2] = add32(m[2], mul32(add32(m[2], 32) >> 5, 5));
            }
        }
    }

    int64_t mid;
    if (w.errlim[c] == 0) {
        int64_t code;
        if (!read_code(bs, high - low, code)) return DEC_EXCEPTION;  // nbits_table[] out of range
        mid = code + low;
    } else if (w.errlim[c] >= 0 && low >= 0 && high >= low && high < ((int64_t)1 << 30)) {
        // The bisection (WordsUtils.cs:486-492) in 32 bits: with a non-negative
        // error limit high-low stays >= 0 and at least halves every step, so it
        // ends within 30 steps and its bits come from one 32-bit look-ahead;
        // branch-free selects instead of a data-dependent branch per bit.
        const int32_t el = w.errlim[c];
        uint32_t lo = (uint32_t)low, hi = (uint32_t)high, md = (hi + lo + 1) >> 1;
        bs.need(32);
        uint32_t look = (uint32_t)bs.win;
        int used = 0;
        while ((int32_t)(hi - lo) > el) {
            const bool one = (look & 1u) != 0;
            look >>= 1;
            used++;
            lo = one ? md : lo;
            hi = one ? hi : md - 1;
            md = (hi + lo + 1) >> 1;
        }
        bs.skip(used);
        mid = (int64_t)md;
        low = (int64_t)lo;
        high = (int64_t)hi;
    } else {
        mid = (high + low + 1) >> 1;
        // The C# loop (WordsUtils.cs:486-492) never ends for some negative error
        // limits (high-low settles in {-2,-1,0}: -1 is a fixed point, 0 waits for a
        // 0 bit, nothing exits below -2): report the exception instead of hanging
        // the lane.  2^24 steps exceed the bits of any block, so no loop that
        // terminates is cut short (the oracle applies the same rule).
        uint32_t steps = 0;
        while (high - low > w.errlim[c]) {
            if (++steps > 72u) {
                const int64_t dd = high - low;
                if ((dd >= -2 && dd <= 0 && (w.errlim[c] <= -3 || dd == -1)) || steps > (1u << 24))
                    return DEC_EXCEPTION;
            }
            if (bs.getbit())
                mid = (high + (low = mid) + 1) >> 1;
            else
                mid = ((high = mid - 1) + low + 1) >> 1;
        }
    }
    const int sign = bs.getbit();
    out = sign ? (int32_t)~(uint32_t)(uint64_t)mid : (int32_t)(uint32_t)(uint64_t)mid;
    if (cb && w.errlim[c] != 0) {
        int64_t code;
        if (!read_code(*cb, high - low, code)) return DEC_EXCEPTION;
        const int64_t value = code + low;
        *corr = (int32_t)(uint32_t)(uint64_t)(sign ? mid - value : value - mid);
    }
    if (flags & HYBRID_BITRATE) {
        int lg = dev_mylog2(mid, exc, tb);
        w.slow[c] = add32(sub32(w.slow[c], add32(w.slow[c], SLO) >> SLS), lg);
    }
    return exc ? DEC_EXCEPTION : DEC_OK;
}

// ---------------------------------------------------------------------------
// decorrelation pass state, sample-major.  Ring semantics: at block frame t
// a 1..8 (or mono negative/0) pass reads slot t&7 and writes (t+(term&7))&7,
// exactly the m/k walk of UnpackUtils.cs:869-899 seen across chunk seams.
// ---------------------------------------------------------------------------
struct PassState {
    int32_t term, delta;
    int32_t wA, wB;
    int32_t rA[8], rB[8];
};

WVF_HD void upd_w(int32_t &w, int32_t s, int32_t b, int32_t delta) {
    if (s != 0 && b != 0) w = ((s ^ b) < 0) ? wvf::sub32(w, delta) : wvf::add32(w, delta);
}
WVF_HD void upd_wc(int32_t &w, int32_t s, int32_t b, int32_t delta) {  // negative terms: clamp +-1024
    if ((s ^ b) < 0) {
        if (s != 0 && b != 0 && (w = wvf::sub32(w, delta)) < -1024) w = w < 0 ? -1024 : 1024;
    } else {
        if (s != 0 && b != 0 && (w = wvf::add32(w, delta)) > 1024) w = w < 0 ? -1024 : 1024;
    }
}

// one stereo frame through one pass (UnpackUtils.cs:688-944 / 946-1154).
// `cont`: the frame is past the first 8 of a call of >= 16 frames, i.e. in
// decorr_stereo_pass_cont -- which only term 0 (a malformed list) notices.
WVF_HD void pass_stereo(PassState &p, uint32_t t, int32_t &L, int32_t &R, bool cont = false) {
    using namespace wvf;
    const int32_t d = p.delta;
    switch (p.term) {
    case 17: {
        int32_t sa = sub32(mul32(2, p.rA[0]), p.rA[1]);
        p.rA[1] = p.rA[0];
        p.rA[0] = add32(apply_weight(p.wA, sa), L);
        upd_w(p.wA, sa, L, d);
        L = p.rA[0];
        int32_t sb = sub32(mul32(2, p.rB[0]), p.rB[1]);
        p.rB[1] = p.rB[0];
        p.rB[0] = add32(apply_weight(p.wB, sb), R);
        upd_w(p.wB, sb, R, d);
        R = p.rB[0];
        break;
    }
    case 18: {
        int32_t sa = sub32(mul32(3, p.rA[0]), p.rA[1]) >> 1;
        p.rA[1] = p.rA[0];
        p.rA[0] = add32(apply_weight(p.wA, sa), L);
        upd_w(p.wA, sa, L, d);
        L = p.rA[0];
        int32_t sb = sub32(mul32(3, p.rB[0]), p.rB[1]) >> 1;
        p.rB[1] = p.rB[0];
        p.rB[0] = add32(apply_weight(p.wB, sb), R);
        upd_w(p.wB, sb, R, d);
        R = p.rB[0];
        break;
    }
    case -1: {
        int32_t sa = add32(L, apply_weight(p.wA, p.rA[0]));
        upd_wc(p.wA, p.rA[0], L, d);
        L = sa;
        int32_t o = add32(R, apply_weight(p.wB, sa));
        upd_wc(p.wB, sa, R, d);
        R = o;
        p.rA[0] = o;
        break;
    }
    case -2: {
        int32_t sb = add32(R, apply_weight(p.wB, p.rB[0]));
        upd_wc(p.wB, p.rB[0], R, d);
        R = sb;
        int32_t o = add32(L, apply_weight(p.wA, sb));
        upd_wc(p.wA, sb, L, d);
        L = o;
        p.rB[0] = o;
        break;
    }
    case -3: {
        int32_t sa = add32(L, apply_weight(p.wA, p.rA[0]));
        upd_wc(p.wA, p.rA[0], L, d);
        int32_t sb = add32(R, apply_weight(p.wB, p.rB[0]));
        upd_wc(p.wB, p.rB[0], R, d);
        p.rB[0] = sa;
        p.rA[0] = sb;
        L = sa;
        R = sb;
        break;
    }
    default: {
        int m = t & 7, k = (t + (p.term & 7)) & 7;
        if (p.term == 0 && cont) {
            // decorr_stereo_pass_cont with term 0 (UnpackUtils.cs:1119-1146): the
            // source is the sample itself; the last 8 outputs become the ring
            int32_t oa = add32(apply_weight(p.wA, L), L);
            upd_w(p.wA, L, L, d);
            int32_t ob = add32(apply_weight(p.wB, R), R);
            upd_w(p.wB, R, R, d);
            p.rA[m] = L = oa;
            p.rB[m] = R = ob;
            break;
        }
        int32_t sa = p.rA[m];
        int32_t oa = add32(apply_weight(p.wA, sa), L);
        upd_w(p.wA, sa, L, d);
        p.rA[k] = oa;
        L = oa;
        int32_t sb = p.rB[m];
        int32_t ob = add32(apply_weight(p.wB, sb), R);
        upd_w(p.wB, sb, R, d);
        p.rB[k] = ob;
        R = ob;
        break;
    }
    }
}

// .wvc (beyond the reference): one stereo frame through one pass, carrying the
// exact-minus-lossy differences cL/cR of the frame along.  The passes keep the
// lossy history and weights (what the encoder decorrelated against); a pass
// whose prediction reads only history moves both channels' exact values by the
// same prediction, so the differences pass through.  Terms -1 and -2 predict
// one channel from the OTHER channel's output of this same pass: the exact
// value predicts from the other channel's exact output, with the same (lossy,
// not yet updated) weight -- the difference changes by the two predictions'
// difference.
WVF_HD void pass_stereo_wvc(PassState &p, uint32_t t, int32_t &L, int32_t &R, int32_t &cL, int32_t &cR,
                            bool cont = false) {
    using namespace wvf;
    const int32_t wA0 = p.wA, wB0 = p.wB;
    pass_stereo(p, t, L, R, cont);
    if (p.term == -1)  // R predicted from this pass's L output
        cR = add32(cR, sub32(apply_weight(wB0, add32(L, cL)), apply_weight(wB0, L)));
    else if (p.term == -2)  // L predicted from this pass's R output
        cL = add32(cL, sub32(apply_weight(wA0, add32(R, cR)), apply_weight(wA0, R)));
}

// one mono value through one pass (UnpackUtils.cs:1156-1240)
WVF_HD void pass_mono(PassState &p, uint32_t t, int32_t &X) {
    using namespace wvf;
    const int32_t d = p.delta;
    if (p.term == 17 || p.term == 18) {
        int32_t sa = p.term == 17 ? sub32(mul32(2, p.rA[0]), p.rA[1]) : (sub32(mul32(3, p.rA[0]), p.rA[1]) >> 1);
        p.rA[1] = p.rA[0];
        p.rA[0] = add32(apply_weight(p.wA, sa), X);
        upd_w(p.wA, sa, X, d);
        X = p.rA[0];
    } else {
        int m = t & 7, k = (t + (p.term & 7)) & 7;
        int32_t sa = p.rA[m];
        int32_t o = add32(apply_weight(p.wA, sa), X);
        upd_w(p.wA, sa, X, d);
        p.rA[k] = o;
        X = o;
    }
}

// ---------------------------------------------------------------------------
// fixup (UnpackUtils.cs:1251-1404): everything except the wvx read is a pure
// per-value map prepared once per block.
// ---------------------------------------------------------------------------
struct Fixup {
    int mode;  // 0 float, 1 int32 per-value (zeros/ones/dups), 2 int32+wvx, 3 plain
    int32_t fshift;
    int32_t zeros, ones, dups, sent_bits, max_width;
    uint32_t mask;
    bool lossy;
    int32_t shift, min_value, max_value, min_shifted, max_shifted;
};

WVF_HD void fixup_init(Fixup &f, const BlockDesc &d) {
    using namespace wvf;
    const uint32_t flags = d.flags;
    f.lossy = (flags & HYBRID_FLAG) != 0;
    int32_t shift = d.shift;
    f.zeros = d.int32_zeros;
    f.ones = d.int32_ones;
    f.dups = d.int32_dups;
    f.sent_bits = d.int32_sent_bits;
    f.max_width = d.int32_max_width;
    f.mask = (uint32_t)shl32(1, f.sent_bits) - 1u;
    f.fshift = d.float_shift;
    if (f.fshift > 32) f.fshift = 32;
    else if (f.fshift < -32) f.fshift = -32;
    if (flags & FLOAT_DATA) {
        f.mode = 0;
    } else if (flags & INT32_DATA) {
        if (d.wvx_state & 0x100) {
            f.mode = 2;
        } else if (f.sent_bits == 0 && (f.zeros + f.ones + f.dups) != 0) {
            f.mode = 1;
            while (f.lossy && (flags & BYTES_STORED) == 3 && shift < 8) {
                if (f.zeros > 0) f.zeros--;
                else if (f.ones > 0) f.ones--;
                else if (f.dups > 0) f.dups--;
                else break;
                shift++;
            }
        } else {
            f.mode = 3;
            shift += f.zeros + f.sent_bits + f.ones + f.dups;
        }
    } else
        f.mode = 3;
    f.shift = shift & 0x1f;
    switch (flags & BYTES_STORED) {
    case 0: f.min_value = sar32(-128, f.shift); f.max_value = sar32(127, f.shift); break;
    case 1: f.min_value = sar32(-32768, f.shift); f.max_value = sar32(32767, f.shift); break;
    case 2: f.min_value = sar32(-8388608, f.shift); f.max_value = sar32(8388607, f.shift); break;
    default: f.min_value = (int32_t)(0x80000000u >> f.shift); f.max_value = sar32(0x7FFFFFFF, f.shift); break;
    }
    f.min_shifted = shl32(f.min_value, f.shift);
    f.max_shifted = shl32(f.max_value, f.shift);
}

// exact float output (OPEN_EXACT_FLOAT) of a FLOAT_DATA block whose descriptor
// asks for it.  Kept apart from Fixup: only the generic kernel's
// decode_pcm_run uses it (the two-wave and pipelined kernels never receive
// such blocks, and their Fixup stays as small as before).
struct XFloat {
    bool on;
    bool wvx;                     // the block carries a wvx stream
    int32_t flags, max_exp, shift;  // ID_FLOAT_INFO's flags, max_exp, shift
};
WVF_HD void xfloat_init(XFloat &x, const BlockDesc &d) {
    x.on = (d.flags & wvf::FLOAT_DATA) && (d.xfloat & XF_ON);
    x.flags = (int32_t)(d.xfloat & 0xffu);
    x.max_exp = (int32_t)((d.xfloat >> 8) & 0xffu);
    x.shift = (int32_t)((d.xfloat >> 16) & 0xffu);
    x.wvx = (d.wvx_state & 1) != 0;
}

WVF_HD int32_t zod(const Fixup &f, int32_t x) {  // zeros / ones / dups (UnpackUtils.cs:1300-1305)
    using namespace wvf;
    if (f.zeros != 0) return shl32(x, f.zeros);
    if (f.ones != 0) return sub32(shl32(add32(x, 1), f.ones), 1);
    if (f.dups != 0) return sub32(shl32(add32(x, x & 1), f.dups), x & 1);
    return x;
}

// everything after the optional wvx read
WVF_HD int32_t fixup_tail(const Fixup &f, int32_t x) {
    using namespace wvf;
    if (f.mode == 0) {  // float_values
        if (f.fshift > 0) x = shl32(x, f.fshift);
        else if (f.fshift < 0) x = sar32(x, -f.fshift);
        if (x > 8388607) x = 8388607;
        else if (x < -8388608) x = -8388608;
        return x;
    }
    if (f.mode == 1) x = zod(f, x);
    if (f.lossy) {
        if (x < f.min_value) return f.min_shifted;
        if (x > f.max_value) return f.max_shifted;
        return shl32(x, f.shift);
    }
    return f.shift ? shl32(x, f.shift) : x;
}

// int32 + wvx (UnpackUtils.cs:1271-1314): reads the extra stream, updates
// crc_x.  The wvx reader has no 0xFF fill: bs_open_read starts it 4 bytes into
// the sub-block while `end` stays at its length (UnpackUtils.cs:130), so a read
// past the payload indexes past the array first -> C# exception (B-10), raised
// through `exc`.  `xlen` = payload bytes after the 4 crc bytes.
WVF_HD int32_t fixup_wvx(const Fixup &f, BitReader &xb, uint32_t xlen, int32_t x, int32_t &crc_x, int &exc) {
    using namespace wvf;
    if (f.sent_bits > 0) {
        int bits_to_read = f.sent_bits;
        bool read = true;
        if (f.max_width > 0) {
            int32_t pvalue = x < 0 ? ~x : x;
            int width = (pvalue ? 32 - __builtin_clz((uint32_t)pvalue) : 0) + f.sent_bits;
            read = width <= f.max_width || (bits_to_read -= width - f.max_width) > 0;
        }
        if (read) {
            if (xb.consumed() + (uint64_t)bits_to_read > 8ull * xlen) exc = 1;
            const uint32_t data = (bits_to_read > 32 ? xb.getbits_big(bits_to_read) : xb.getbits_reg(bits_to_read)) & f.mask;
            x = shl32((int32_t)((uint32_t)shl32(x, bits_to_read) | data), f.sent_bits - bits_to_read);
        } else
            x = shl32(x, f.sent_bits);
    }
    x = zod(f, x);
    crc_x = add32(add32(mul32(crc_x, 9), mul32(x & 0xffff, 3)), (x >> 16) & 0xffff);
    return fixup_tail(f, x);
}

// Exact float output (OPEN_EXACT_FLOAT; beyond the reference):
// WavPack 4's float_values, where FloatUtils.cs:32-56 scales to 24-bit
// integers instead.  A nonzero integer is the float's mantissa (implicit bit
// included) shifted right by float_max_exp - exponent; the wvx stream, when
// the block carries one, holds the bits that shift dropped (FLOAT_SHIFT_*),
// the floats that became 0 (FLOAT_ZEROS_SENT / FLOAT_NEG_ZEROS) and inf/nan
// mantissas (FLOAT_EXCEPTIONS: integer +-2^24).  Returns the float's bits;
// crc_x takes crc * 27 + mantissa * 9 + exponent * 3 + sign per value (the wvx
// header's crc).  A read past the wvx payload, or a shift no encoder makes,
// sets `bad` (the block's CRC verdict then fails).
WVF_HD int32_t fixup_xfloat(const XFloat &f, BitReader &xb, uint32_t xlen, int32_t x, int32_t &crc_x, int &bad) {
    using namespace wvf;
    const bool wx = f.wvx;
    uint32_t sign = 0, exp = (uint32_t)f.max_exp, mant = 0;
    if (x == 0) {
        exp = 0;
        if (wx && (f.flags & FLOAT_ZEROS_SENT)) {
            if (xb.getbit()) {  // a float the shift took to 0: sent whole
                mant = xb.getbits(23);
                if (f.max_exp >= 25) exp = xb.getbits(8);
                sign = (uint32_t)xb.getbit();
            } else if (f.flags & FLOAT_NEG_ZEROS) {
                sign = (uint32_t)xb.getbit();
            }
        } else if (wx && (f.flags & FLOAT_NEG_ZEROS)) {
            sign = (uint32_t)xb.getbit();
        }
    } else {
        uint32_t v = (uint32_t)shl32(x, f.shift);
        if ((int32_t)v < 0) {
            v = 0u - v;
            sign = 1;
        }
        if (wx && v == 0x1000000u) {  // inf / nan
            if (xb.getbit()) mant = xb.getbits(23);
            exp = 255;
        } else if (!wx && v >= 0x1000000u) {
            while (v & 0xf000000u) {
                v >>= 1;
                ++exp;
            }
            mant = v;
        } else {
            int sc = 0;
            if (exp)
                while (!(v & 0x800000u) && --exp) {
                    sc++;
                    v <<= 1;
                }
            if (sc > 23) {
                bad = 1;
            } else if (sc) {
                const uint32_t m = (1u << sc) - 1u;
                if ((f.flags & FLOAT_SHIFT_ONES) || (wx && (f.flags & FLOAT_SHIFT_SAME) && xb.getbit()))
                    v |= m;
                else if (wx && (f.flags & FLOAT_SHIFT_SENT))
                    v |= xb.getbits(sc) & m;
            }
            mant = v;
        }
    }
    mant &= 0x7fffffu;
    exp &= 0xffu;
    if (wx && xb.consumed() > 8ull * xlen) bad = 1;
    crc_x = add32(add32(add32(mul32(crc_x, 27), mul32((int32_t)mant, 9)), mul32((int32_t)exp, 3)), (int32_t)sign);
    return (int32_t)((sign << 31) | (exp << 23) | mant);
}

// ---------------------------------------------------------------------------
// one PCM block.  PcmState is the part of the WavpackStream a decode adapts:
// pcm_state_load fills it from the descriptor and, inside a chain, keeps what
// the block did not re-send from the decode before it (Appendix B-8).
// ---------------------------------------------------------------------------
struct PcmState {
    BitReader bs, xb;
    BitReader cb;         // .wvc correction stream (d.wvc_len > 0)
    bool wvc;
    Entropy w;
    PassState ps[MAXP];
    int32_t crc, crc_x;   // wps.crc / wps.crc_x
    bool muted;           // wps.mute_error
    bool crc_garbage;     // the running crc went over stale buffer contents
    bool pass_garbage;    // a pass ran over stale residuals (get_words stopped short)
    bool xbad;            // exact float: the wvx stream ran out or held an impossible value
};

// Every reference pass call leaves its ring rotated so that slot 0 is the
// oldest value (UnpackUtils.cs:920-936, 1139-1146, 1225-1233); sample-major
// decoding keeps value t in slot t & 7 instead, t counting the frames the
// passes ran over in the block.  Rotating by t gives the reference's layout.
WVF_HD bool ring_term(int term, bool mono) { return mono ? (term != 17 && term != 18) : (term >= 0 && term <= 8); }
WVF_HD void ring_normalize(PassState &p, uint32_t t, bool mono) {
    const int r = (int)(t & 7u);
    if (!r) return;
    int32_t a[8], b[8];
    for (int k = 0; k < 8; k++) {
        a[k] = p.rA[(r + k) & 7];
        b[k] = p.rB[(r + k) & 7];
    }
    for (int k = 0; k < 8; k++) {
        p.rA[k] = a[k];
        if (!mono) p.rB[k] = b[k];  // decorr_mono_pass rotates samples_A only
    }
}

// the block's starting state: the descriptor's values, except what d.inherit /
// d.inherit_passes take from `s` as the previous decode left it.  Returns the
// status bits that follow from the carried state (ST_NONDET).
WVF_HD uint32_t pcm_state_load(PcmState &s, const BlockDesc &d, const uint8_t *blob) {
    const uint32_t inh = d.inherit;
    uint32_t status = 0;
    if (!(inh & INH_BITS)) {
        s.bs.init(blob, d.bits_off, d.bits_len);
    } else if (!(inh & INH_NOINIT)) {
        // unpack_init clears the register but not its bit count (UnpackUtils.cs:34):
        // the rest of the current byte reads as zeros
        s.bs.win &= ~((1ull << (s.bs.nb & 7)) - 1ull);
    }
    s.wvc = d.wvc_len > 0;
    if (s.wvc) s.cb.init(blob, d.wvc_off, d.wvc_len);
    if (!(inh & INH_WVX)) {
        s.xb.init(blob, d.wvx_off, d.wvx_len);
        if (d.wvx_state & 0x100) {
            int skip = (d.wvx_state >> 1) & 0x7f;
            if (skip) s.xb.getbits(skip);
        }
    }
    Entropy &w = s.w;
    if (!(inh & INH_ENTROPY)) {
        for (int c = 0; c < 2; c++) {
            for (int k = 0; k < 3; k++) w.med[c][k] = d.median[c][k];
            w.slow[c] = d.slow_level[c];
            w.errlim[c] = 0;
            w.acc[c] = d.bitrate_acc[c];
            w.dlt[c] = d.bitrate_delta[c];
        }
        w.zeros_acc = 0;
        w.h0 = w.h1 = 0;
    } else {  // read_hybrid_profile without read_entropy_vars: those fields only
        for (int c = 0; c < 2; c++) {
            if (!(inh & (INH_SLOW0 << c))) w.slow[c] = d.slow_level[c];
            if (!(inh & (INH_ACC0 << c))) w.acc[c] = d.bitrate_acc[c];
            if (!(inh & (INH_DLT0 << c))) w.dlt[c] = d.bitrate_delta[c];
        }
    }
    bool fresh_passes = true;
    for (int i = 0; i < d.num_terms && i < MAXP; i++) {
        PassState &p = s.ps[i];
        p.term = d.term[i];
        p.delta = d.delta[i];
        if ((d.inherit_passes >> i) & 1u) {
            fresh_passes = false;
        } else {
            p.wA = d.weight_A[i];
            p.wB = d.weight_B[i];
        }
        if ((d.inherit_passes >> (16 + i)) & 1u) {
            fresh_passes = false;
        } else {
            for (int k = 0; k < 8; k++) {
                p.rA[k] = d.samples_A[i][k];
                p.rB[k] = d.samples_B[i][k];
            }
        }
    }
    if (fresh_passes) s.pass_garbage = false;
    else if (s.pass_garbage) status |= ST_NONDET;  // carried from passes over stale residuals
    if (!(inh & INH_NOINIT)) {  // unpack_init (UnpackUtils.cs:32-33)
        s.crc = s.crc_x = -1;
        s.muted = false;
        s.crc_garbage = false;
        s.xbad = false;
    }
    return status;
}

// The block's frames from state `s`.  CHAIN: leave `s` as the reference's
// stream is left for the next block -- the muting chunk's remaining words and
// passes still run (UnpackUtils.cs:556-607 precede the mute test), and the
// rings end in the reference's layout.
template <class Store, bool CHAIN>
WVF_HD uint32_t decode_pcm_run(PcmState &s, const BlockDesc &d, Store &out, uint32_t *exc_frame) {
    using namespace wvf;
    const uint32_t flags = d.flags;
    const bool mono = (flags & MONO_DATA) != 0;       // decode path (UnpackUtils.cs:549)
    const bool mono_out = (flags & MONO_FLAG) != 0;   // ints written per frame: 1 or 2
    const bool fstereo = (flags & FALSE_STEREO) != 0;
    const bool joint = (flags & JOINT_STEREO) != 0;
    const int32_t ml = d.mute_limit;
    const int nt = d.num_terms;
    const uint32_t nfr = d.nframes;
    const int och = mono_out ? 1 : 2;
    // where a call's values land (UnpackUtils.cs:510-686 writes `wch` ints a frame from the
    // call's buffer position; the caller advances out_nch a frame, WavPackUtils.cs:263-268):
    // wch = 1 for MONO_FLAG without FALSE_STEREO, else 2 (FALSE_STEREO's copy, :655-664).
    // When they differ, a 2-int block in a 1-int file shows the first n of its 2n ints
    // (the next block of the call writes over the rest, or the call ends there; the
    // framing raises the call's exception when 2n pass the caller's buffer), and a 1-int
    // block in a 2-int file fills the first n of its 2n slots (the rest keep the caller's
    // stale buffer: ST_NONDET from the framing)
    // (a call that starts muted zero-fills MONO_FLAG ? n : 2n ints and returns before the
    // FALSE_STEREO copy, :527-543: width och)
    const uint32_t wch = (mono_out && !fstereo) ? 1u : 2u, sch = d.out_nch;
    auto store = [&](uint32_t wch, uint32_t f0, uint32_t j, uint32_t n, int32_t a, int32_t b) {
        if (wch == sch) {
            const uint64_t o = (uint64_t)(f0 + j) * sch;
            out.put(o, a);
            if (wch == 2) out.put(o + 1, b);
        } else if (wch == 2) {  // sch == 1
            const uint32_t p = 2u * j;
            if (p < n) out.put((uint64_t)f0 + p, a);
            if (p + 1u < n) out.put((uint64_t)f0 + p + 1u, b);
        } else {  // wch == 1, sch == 2
            out.put((uint64_t)f0 * 2u + j, a);
        }
    };
    BitReader &bs = s.bs;
    BitReader &xb = s.xb;
    Entropy &w = s.w;
    PassState *ps = s.ps;

    Fixup fx;
    fixup_init(fx, d);
    XFloat xf;
    xfloat_init(xf, d);

    uint32_t status = 0;
    if (fstereo && fx.mode == 2) status |= ST_NONDET;  // fixup reads wvx bits for 2n values (n stale)
    uint32_t f = 0;   // block frame index (also the ring clock)
    uint32_t tp = 0;  // frames the passes ran over (CHAIN)
    uint32_t chunk_len = d.first_chunk;
    uint32_t bsp = d.first_bsp;
    bool first = true;
    while (f < nfr) {
        uint32_t n = chunk_len;
        if (n > nfr - f) n = nfr - f;
        if (s.muted) {  // mute_error set: unpack_samples zero-fills (UnpackUtils.cs:527-543)
            for (uint32_t j = 0; j < n; j++) store((uint32_t)och, f, j, n, 0, 0);
            f += n;
            chunk_len = next_call_len(d, f);
            bsp = 0;
            first = false;
            continue;
        }
        // state at the chunk start, for the wvx rewind on muting
        BitReader xb0 = xb;
        int32_t crcx0 = s.crc_x;
        bool crc_stop = false;
        int mute_at = -1;  // chunk-relative frame that mutes the chunk
        bool words_short = false;
        for (uint32_t j = 0; j < n; j++) {
            uint32_t t = f + j;
            int32_t L, R = 0, cL = 0, cR = 0;
            BitReader *cbp = s.wvc ? &s.cb : nullptr;
            int rc = get_word(w, bs, flags, 0, true, L, MemTabs(), cbp, &cL);
            if (rc == DEC_OK && !mono) rc = get_word(w, bs, flags, 1, false, R, MemTabs(), cbp, &cR);
            if (rc != DEC_OK) {
                if (rc == DEC_EXCEPTION) {
                    if (exc_frame) *exc_frame = t;  // block frame of the word that threw
                    return status | ST_EXCEPTION;
                }
                // get_words stopped short: the reference decorrelates stale buffer
                // contents; the chunk is muted and the CRC is garbage (-> error)
                status |= ST_BITS_ERROR;
                if (mono && first && bsp > 0) status |= ST_NONDET;
                mute_at = (int)j;
                s.crc_garbage = true;  // the verdict at block end is "error" (w.p. 1 - 2^-32)
                words_short = true;
                break;
            }
            if (mono) {
                for (int i = 0; i < nt; i++) pass_mono(ps[i], t, L);
                L = add32(L, cL);  // .wvc: the exact value (the passes keep the lossy history)
                int32_t a = L < 0 ? (int32_t)(0u - (uint32_t)L) : L;
                if (!crc_stop && a > ml) {
                    uint32_t q = bsp + j;  // absolute buffer index (quirk B-6)
                    if (q != n) {
                        mute_at = (int)j;
                        break;
                    }
                    crc_stop = true;
                }
                if (!crc_stop) s.crc = add32(mul32(s.crc, 3), L);
            } else {
                if (s.wvc) {  // .wvc: the exact values (pass_stereo_wvc)
                    for (int i = 0; i < nt; i++) pass_stereo_wvc(ps[i], t, L, R, cL, cR, n >= 16 && j >= 8);
                    L = add32(L, cL);
                    R = add32(R, cR);
                } else {
                    for (int i = 0; i < nt; i++) pass_stereo(ps[i], t, L, R, n >= 16 && j >= 8);
                }
                if (joint) {
                    R = sub32(R, L >> 1);
                    L = add32(L, R);
                }
                int32_t a = L < 0 ? (int32_t)(0u - (uint32_t)L) : L;
                int32_t b = R < 0 ? (int32_t)(0u - (uint32_t)R) : R;
                if (a > ml || b > ml) {
                    mute_at = (int)j;
                    break;
                }
                s.crc = add32(mul32(add32(mul32(s.crc, 3), L), 3), R);
            }
            // (short) weight stores at the pass-call seams (B-4)
            if ((!mono && n >= 16 && j == 7) || j == n - 1) {
                for (int i = 0; i < nt; i++) {
                    ps[i].wA = (int16_t)ps[i].wA;
                    ps[i].wB = (int16_t)ps[i].wB;
                }
            }
            // fixup + store
            int32_t oL, oR;
            if (fx.mode == 2) {
                int xexc = 0;
                oL = fixup_wvx(fx, xb, d.wvx_len, L, s.crc_x, xexc);
                oR = mono ? 0 : fixup_wvx(fx, xb, d.wvx_len, R, s.crc_x, xexc);
                if (xexc) {  // fixup_samples of this call threw (the call's frame)
                    if (exc_frame) *exc_frame = t;
                    return status | ST_EXCEPTION;
                }
            } else if (xf.on) {
                int bad = 0;
                oL = fixup_xfloat(xf, xb, d.wvx_len, L, s.crc_x, bad);
                oR = mono ? 0 : fixup_xfloat(xf, xb, d.wvx_len, R, s.crc_x, bad);
                if (bad) s.xbad = true;
            } else {
                oL = fixup_tail(fx, L);
                oR = mono ? 0 : fixup_tail(fx, R);
            }
            store(wch, f, j, n, oL, fstereo ? oL : oR);
        }
        if (CHAIN && mute_at >= 0) {
            if (words_short) {
                s.pass_garbage = nt > 0;  // the passes ran over the chunk's stale residuals
            } else {
                // the rest of the chunk's words and passes (their values are discarded)
                for (uint32_t j = (uint32_t)mute_at; j < n; j++) {
                    const uint32_t t = f + j;
                    if (j > (uint32_t)mute_at) {
                        int32_t L, R = 0;
                        int rc = get_word(w, bs, flags, 0, true, L);
                        if (rc == DEC_OK && !mono) rc = get_word(w, bs, flags, 1, false, R);
                        if (rc == DEC_EXCEPTION) {
                            if (exc_frame) *exc_frame = t;
                            return status | ST_EXCEPTION;
                        }
                        if (rc != DEC_OK) {
                            status |= ST_BITS_ERROR;
                            s.pass_garbage = nt > 0;
                            break;
                        }
                        if (mono) {
                            for (int i = 0; i < nt; i++) pass_mono(ps[i], t, L);
                        } else {
                            for (int i = 0; i < nt; i++) pass_stereo(ps[i], t, L, R, n >= 16 && j >= 8);
                        }
                    }
                    if ((!mono && n >= 16 && j == 7) || j == n - 1) {
                        for (int i = 0; i < nt; i++) {
                            ps[i].wA = (int16_t)ps[i].wA;
                            ps[i].wB = (int16_t)ps[i].wB;
                        }
                    }
                }
            }
        }
        tp = f + n;
        if (mute_at >= 0) {
            // UnpackUtils.cs:649-664: zero the whole chunk, then fixup_samples runs on
            // the zeros (which is not always 0: int32 'ones', wvx reads)
            status |= ST_MUTED;
            s.muted = true;
            xb = xb0;
            s.crc_x = crcx0;
            for (uint32_t j = 0; j < n; j++) {
                int32_t z0, z1 = 0;
                if (fx.mode == 2) {
                    int xexc = 0;
                    z0 = fixup_wvx(fx, xb, d.wvx_len, 0, s.crc_x, xexc);
                    if (!mono) z1 = fixup_wvx(fx, xb, d.wvx_len, 0, s.crc_x, xexc);
                    if (xexc) {
                        if (exc_frame) *exc_frame = f + j;
                        return status | ST_EXCEPTION;
                    }
                } else if (xf.on) {
                    z0 = 0;  // +0.0f; the wvx stream is not read past a mute
                } else {
                    z0 = fixup_tail(fx, 0);
                    z1 = mono ? 0 : fixup_tail(fx, 0);
                }
                store(wch, f, j, n, z0, fstereo ? z0 : z1);
            }
        }
        f += n;
        chunk_len = next_call_len(d, f);
        bsp = 0;
        first = false;
    }
    if (CHAIN)
        for (int i = 0; i < nt; i++)
            if (ring_term(ps[i].term, mono)) ring_normalize(ps[i], tp, mono);
    if (nfr == d.block_samples) {  // check_crc_error at block end (WavPackUtils.cs:273-275)
        status |= ST_CRC_CHECKED;
        bool err = s.crc_garbage || s.crc != d.crc;
        if (!(flags & FLOAT_DATA) && (d.wvx_state & 1) && s.crc_x != d.crc_mvx) err = true;
        if (xf.on && (s.xbad || ((d.wvx_state & 1) && s.crc_x != d.crc_mvx))) err = true;
        if (err) status |= ST_CRC_ERROR;
    }
    return status;
}

// one block from its descriptor alone, its state in `s` (the device kernel passes a
// wave's LDS copy: the pass rings and weights are indexed by run-time pass and slot
// numbers, which in registers would live in scratch memory)
template <class Store>
WVF_HD uint32_t decode_pcm_block_in(PcmState &s, const BlockDesc &d, const uint8_t *blob, Store &out,
                                    uint32_t *exc_frame = nullptr) {
    pcm_state_load(s, d, blob);
    return decode_pcm_run<Store, false>(s, d, out, exc_frame);
}
template <class Store>
WVF_HD uint32_t decode_pcm_block(const BlockDesc &d, const uint8_t *blob, Store &out, uint32_t *exc_frame = nullptr) {
    PcmState s;
    return decode_pcm_block_in(s, d, blob, out, exc_frame);
}

// ---------------------------------------------------------------------------
// one DSD block (DsdUtils.cs:56-136 with decode_fast :244-304 and
// decode_high :391-493).  Muting fills 0x55 from the *call* buffer start
// (quirk B-9); the kernel only records where muting began (ST_DSD_MUTE +
// the returned chunk index) and a post-pass writes the fills in block order.
// `ptable` is 256 ints of per-block scratch for mode 3.
// ---------------------------------------------------------------------------
struct DsdResult {
    uint32_t status;
    uint32_t mute_chunk;  // first muted chunk (valid with ST_DSD_MUTE)
};

// init_ptable (DsdUtils.cs:321-341; rate_s is 20, the framing rejects any
// other): mode 3's starting probability table from the block's rate_i.  A
// uniform serial recurrence of at most 3,469 steps over all 256 rate_i (value
// reaches 0x10000 and stops moving, which ends the rate growth); of `nl` lanes,
// lane `lane` stores entries i and 255 - i for i == lane (mod nl).
WVF_HD void dsd_ptable_init(int32_t rate_i, int32_t *pt, uint32_t lane, uint32_t nl) {
    int32_t value = 0x808000, rate = rate_i << 8;
    for (int32_t c = (rate + 128) >> 8; c > 0; c--) value += (0x00010000 - value) >> 8;
    for (uint32_t i = 0; i < 128; ++i) {
        if (i % nl == lane) {
            pt[i] = value;
            pt[255 - i] = 0x100ffff - value;
        }
        if (value > 0x010000) {
            rate += (rate * 20 + 128) >> 8;
            for (int32_t c = (rate + 64) >> 7; c > 0; c--) value += (0x00010000 - value) >> 8;
        }
    }
}

// The DSD decode state of WavpackStream.dsds (and the crc / mute_error unpack_init
// resets): per block from its descriptor, or -- a block without ID_DSD_BLOCK, or a
// header read without unpack_init (DsdUtils.cs:17-54, UnpackUtils.cs:24-68,
// WavPackUtils.cs:219-251) -- carried on from the block decoded before it (a chain,
// chain_blocks in wv_framing.cpp; Appendix B-8 for DSD).
struct DsdState {
    const uint8_t *data;  // the metadata sub-block the bytes come from, from its payload start
    uint32_t dlen, bp;    // its bytes from there (data.Length - byteptr at the payload start), bytes read
    uint32_t kind;        // the mode (KIND_DSD_*) of the sub-block
    // mode 1 (init_dsd_block_fast's tables, host-built)
    int bins;
    const uint8_t *prob;
    const uint16_t *summed;
    const uint8_t *lookup;
    const int32_t *vlook;
    uint32_t low, high, value;
    int p0, p1;
    // mode 3 (the ptable itself lives in the caller's 256-int scratch)
    int32_t F[2][9];  // value, filter0..6, factor
    int32_t bytei[2];
    int32_t crc;
    bool mute;
};

// the state init_dsd_block leaves for block d (ptable: 256 ints of scratch, mode 3)
WVF_HD void dsd_state_init(DsdState &S, const BlockDesc &d, const uint8_t *blob, const uint8_t *tables,
                           int32_t *ptable, const int32_t *ptables_all) {
    S.data = blob + d.bits_off;  // data[byteptr] with byteptr == 0 here
    S.dlen = d.dsd_data_len;
    S.bp = 0;
    S.kind = d.kind;
    S.bins = d.dsd_history_bins;
    S.prob = tables + d.dsd_table_off;
    S.summed = (const uint16_t *)(tables + d.dsd_table_off + (size_t)S.bins * 256);
    S.lookup = tables + d.dsd_table_off + (size_t)S.bins * 768;
    S.vlook = (const int32_t *)(tables + d.dsd_table_off + (size_t)S.bins * 2048);
    S.low = 0;
    S.high = 0xFFFFFFFFu;
    S.value = 0;
    S.p0 = S.p1 = 0;
    S.bytei[0] = S.bytei[1] = 0;
    S.crc = -1;
    S.mute = false;
    if (d.kind == KIND_DSD_FAST || d.kind == KIND_DSD_HIGH) {
        for (int i = 0; i < 4; i++) S.value = (S.value << 8) | S.data[S.bp++];
    }
    if (d.kind == KIND_DSD_HIGH) {
        if (ptables_all) {  // the device's precomputed rows (g_dsd_ptables)
            const int32_t *pt0 = ptables_all + (uint32_t)(d.dsd_rate_i & 255) * 256u;
            for (int i = 0; i < 256; i++) ptable[i] = pt0[i];
        } else {
            dsd_ptable_init(d.dsd_rate_i, ptable, 0, 1);
        }
        for (int c = 0; c < 2; c++) {
            S.F[c][0] = 0;
            S.F[c][1] = 0;
            for (int k = 0; k < 5; k++) S.F[c][2 + k] = d.dsd_filters[c][k];
            S.F[c][7] = 0;  // filter6
            S.F[c][8] = d.dsd_filters[c][5];  // factor
        }
    }
}

// block d's calls (unpack_dsd_samples, DsdUtils.cs:56-136) from state S; d's own
// header gives the layout, the frames and the crc to check
template <class Store>
WVF_HD DsdResult dsd_run(DsdState &S, const BlockDesc &d, int32_t *ptable, Store &out) {
    using namespace wvf;
    const uint32_t flags = d.flags;
    const bool mono = (flags & MONO_DATA) != 0;
    const bool fstereo = (flags & FALSE_STEREO) != 0;
    const int wch = mono ? 1 : 2;
    const int och = (flags & MONO_FLAG) ? 1 : 2;
    const uint8_t *data = S.data;
    const uint32_t dlen = S.dlen;
    uint32_t bp = S.bp;
    int32_t crc = S.crc;
    DsdResult res = {0, 0};
    bool mute = S.mute;
    const int bins = S.bins;
    const uint8_t *prob = S.prob;
    const uint16_t *summed = S.summed;
    const uint8_t *lookup = S.lookup;
    const int32_t *vlook = S.vlook;
    uint32_t low = S.low, high = S.high, value = S.value;
    int p0 = S.p0, p1 = S.p1;
    int32_t(&F)[2][9] = S.F;
    int32_t *bytei = S.bytei;
    const uint32_t kind = S.kind;

    uint32_t f = 0, chunk_len = d.first_chunk, ci = 0;
    while (f < d.nframes) {
        uint32_t n = chunk_len;
        if (n > d.nframes - f) n = d.nframes - f;
        bool chunk_ok = true;
        if (!mute) {
            for (uint32_t j = 0; j < n && chunk_ok; j++) {
                int32_t v[2] = {0, 0};
                bool past[2] = {false, false};
                for (int c = 0; c < wch; c++) {
                    int code;
                    if (kind == KIND_DSD_RAW) {
                        // (past the sub-block the reference clamps the count, DsdUtils.cs:73-82:
                        // neither the caller's buffer nor the crc sees those values -- the
                        // buffer keeps what it held; only a block continuing a consumed one
                        // gets there)
                        past[c] = bp >= dlen;
                        if (past[c]) res.status |= ST_NONDET;
                        code = bp < dlen ? data[bp] : 0;
                        bp++;
                    } else if (kind == KIND_DSD_FAST) {
                        const int pi = p0 * 256;
                        uint32_t tot = summed[pi + 255];
                        if (tot == 0) { chunk_ok = false; break; }
                        uint32_t mult = (high - low) / tot;
                        if (mult == 0) {
                            if (dlen - bp >= 4)
                                for (int i = 0; i < 4; i++) value = (value << 8) | data[bp++];
                            low = 0;
                            high = 0xFFFFFFFFu;
                            mult = high / tot;
                            if (mult == 0) { chunk_ok = false; break; }
                        }
                        uint32_t index = (value - low) / mult;
                        if (index >= tot) { chunk_ok = false; break; }
                        code = lookup[vlook[p0] + index];
                        if (code > 0) low += summed[pi + code - 1] * mult;
                        high = low + prob[pi + code] * mult - 1;
                        if (mono)
                            p0 = code & (bins - 1);
                        else {
                            p0 = p1;
                            p1 = code & (bins - 1);
                        }
                        while (((high ^ low) & 0xFF000000u) == 0 && bp < dlen) {
                            value = (value << 8) | data[bp++];
                            high = (high << 8) | 0xFF;
                            low <<= 8;
                        }
                    } else {
                        code = 0;  // filled below for both channels at once
                    }
                    v[c] = code;
                }
                if (!chunk_ok) break;
                if (kind == KIND_DSD_HIGH) {
                    for (int c = 0; c < wch; c++) F[c][0] = add32(sub32(F[c][2], F[c][6]), mul32(F[c][7], F[c][8]) >> 2);
                    for (int bit = 0; bit < 8; bit++) {
                        for (int c = 0; c < wch; c++) {
                            int32_t *q = F[c];
                            int pp = (q[0] >> 8) & 255;
                            uint32_t split = low + ((high - low) >> 8) * ((uint32_t)ptable[pp] >> 16);
                            if (value <= split) {
                                high = split;
                                ptable[pp] += (0x010000FE - ptable[pp]) >> 8;
                                q[1] = -1;
                            } else {
                                low = split + 1;
                                ptable[pp] += (0x00010000 - ptable[pp]) >> 8;
                                q[1] = 0;
                            }
                            while (((high ^ low) & 0xFF000000u) == 0 && bp < dlen) {
                                value = (value << 8) | data[bp++];
                                high = (high << 8) | 0xFF;
                                low <<= 8;
                            }
                            q[0] = add32(q[0], mul32(q[7], 8));
                            bytei[c] = shl32(bytei[c], 1) | (q[1] & 1);
                            q[8] = add32(q[8], (((q[0] ^ q[1]) >> 31) | 1) & ((q[0] ^ sub32(q[0], mul32(q[7], 16))) >> 31));
                            q[2] = add32(q[2], sub32(q[1] & (1 << 20), q[2]) >> 6);
                            q[3] = add32(q[3], sub32(q[1] & (1 << 20), q[3]) >> 4);
                            q[4] = add32(q[4], sub32(q[3], q[4]) >> 4);
                            q[5] = add32(q[5], sub32(q[4], q[5]) >> 4);
                            q[0] = sub32(q[5], q[6]) >> 4;
                            q[6] = add32(q[6], q[0]);
                            q[7] = add32(q[7], sub32(q[0], q[7]) >> 3);
                            q[0] = add32(sub32(q[2], q[6]), mul32(q[7], q[8]) >> 2);
                        }
                    }
                    for (int c = 0; c < wch; c++) {
                        v[c] = bytei[c] & 0xFF;
                        F[c][8] = sub32(F[c][8], add32(F[c][8], 512) >> 10);
                    }
                }
                for (int c = 0; c < wch; c++)
                    if (!past[c]) crc = add32(crc, add32(shl32(crc, 1), v[c]));
                uint64_t o = (uint64_t)(f + j) * och;
                if (mono && !fstereo) {
                    if (!past[0]) out.put(o, v[0]);
                } else if (fstereo) {
                    if (!past[0]) {
                        out.put(o, v[0]);
                        out.put(o + 1, v[0]);
                    }
                } else {
                    if (!past[0]) out.put(o, v[0]);
                    if (!past[1]) out.put(o + 1, v[1]);
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
    S.bp = bp;
    S.crc = crc;
    S.mute = mute;
    S.low = low;
    S.high = high;
    S.value = value;
    S.p0 = p0;
    S.p1 = p1;
    return res;
}

template <class Store>
WVF_HD DsdResult decode_dsd_block(const BlockDesc &d, const uint8_t *blob, const uint8_t *tables, int32_t *ptable,
                                  Store &out, const int32_t *ptables_all = nullptr) {
    DsdState S;
    dsd_state_init(S, d, blob, tables, ptable, ptables_all);
    return dsd_run(S, d, ptable, out);
}

// a block of a DSD chain: the head starts from its descriptor, a member continues S
// (unpack_init's crc / mute reset unless its header was read without unpack_init)
template <class Store>
WVF_HD DsdResult decode_dsd_chained(DsdState &S, const BlockDesc &d, bool head, const uint8_t *blob,
                                    const uint8_t *tables, int32_t *ptable, Store &out,
                                    const int32_t *ptables_all = nullptr) {
    if (head) {
        dsd_state_init(S, d, blob, tables, ptable, ptables_all);
    } else if (!(d.inherit & INH_NOINIT)) {
        S.crc = -1;
        S.mute = false;
    }
    return dsd_run(S, d, ptable, out);
}

}  // namespace wvg
