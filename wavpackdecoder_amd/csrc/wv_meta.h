// wv_meta.h -- the metadata value readers, shared by the device parse kernel
// and the host framing ("device-side metadata parse").
//
// The host framing walks every block's sub-blocks (ids, lengths, the checks
// that decide whether unpack_init succeeds: UnpackUtils.cs:24-68) but leaves
// the *values* of four readers to the device:
//   read_decorr_weights   UnpackUtils.cs:196-239
//   read_decorr_samples   UnpackUtils.cs:250-360 (quirk B-7: every pass is
//                         filled with the last pass's term layout)
//   read_entropy_vars     WordsUtils.cs:75-116
//   read_hybrid_profile   WordsUtils.cs:124-187
// Each deferred read becomes a MetaItem (where its bytes are plus the stream
// state it depends on).  A block's descriptor carries the items still pending
// when it is snapshotted (a MetaJob); `wv_meta_parse` (one lane per job)
// applies them, in stream order, to the descriptor the host uploaded.  The
// host defers a read only when the value computation cannot fail and reads
// nothing past the sub-block's byte_length (so the bytes in the batch blob are
// exactly what the C# reader sees); every other read runs on the host, after
// the pending items were applied there (`meta_apply` on the host state).
#pragma once
#include <stdint.h>

#include "wv_decode_core.h"
#include "wv_desc.h"
#include "wv_format.h"

namespace wvg {

enum MetaKind : uint32_t { META_WEIGHTS = 1, META_SAMPLES = 2, META_ENTROPY = 3, META_HYBRID = 4 };

struct MetaItem {
    uint64_t off;       // sub-block data: blob offset (device) / file offset (host framing)
    uint32_t kind;      // MetaKind
    uint32_t len;       // byte_length
    int32_t num_terms;  // passes in the stream when the reader ran
    int32_t arg;        // WEIGHTS: termcnt; SAMPLES: the quirk term; HYBRID: header flags
    int32_t counter0;   // SAMPLES: first byte (v0x402 hybrid skips 2/4)
    uint32_t mono;      // header flags & MONO_DATA
};
static_assert(sizeof(MetaItem) == 32, "MetaItem layout");

struct MetaJob {
    uint32_t desc;   // descriptor index in the batch
    uint32_t first;  // first item in the batch item array
    uint32_t count;  // items, applied in order
    uint32_t pad_;
};

// The values the four readers produce, with the BlockDesc field names: V is a
// BlockDesc (device) or the host framing's staging copy.
template <class V>
WVF_HD void meta_apply(V &v, const MetaItem &it, const uint8_t *base) {
    const uint8_t *p = base + it.off;
    const bool mono = it.mono != 0;
    int exc = 0;  // exp2s of a 16-bit value never reaches int.MinValue
    auto u16 = [&](int o) -> int32_t { return (int32_t)p[o] | ((int32_t)p[o + 1] << 8); };
    auto s16 = [&](int o) -> int32_t { return (int32_t)(int16_t)(uint16_t)u16(o); };
    if (it.kind == META_WEIGHTS) {
        // the last `termcnt` passes, from num_terms - 1 down (UnpackUtils.cs:211-236)
        int counter = 0;
        for (int k = 0; k < it.arg; k++) {
            const int idx = it.num_terms - 1 - k;
            v.weight_A[idx] = (int16_t)wvf::restore_weight((int8_t)p[counter++]);
            v.weight_B[idx] = mono ? (int16_t)0 : (int16_t)wvf::restore_weight((int8_t)p[counter++]);
        }
    } else if (it.kind == META_SAMPLES) {
        for (int i = 0; i < it.num_terms; i++)
            for (int m = 0; m < 8; m++) v.samples_A[i][m] = v.samples_B[i][m] = 0;
        const int term = it.arg;
        int32_t tA[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tB[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int counter = it.counter0, idx = it.num_terms - 1;
        while (counter < (int)it.len) {
            if (term > wvf::MAX_TERM) {
                tA[0] = dev_exp2s(s16(counter), exc);
                tA[1] = dev_exp2s(s16(counter + 2), exc);
                counter += 4;
                if (!mono) {
                    tB[0] = dev_exp2s(s16(counter), exc);
                    tB[1] = dev_exp2s(s16(counter + 2), exc);
                    counter += 4;
                }
            } else if (term < 0) {
                tA[0] = dev_exp2s(s16(counter), exc);
                tB[0] = dev_exp2s(s16(counter + 2), exc);
                counter += 4;
            } else {
                for (int m = 0; m < term; m++) {
                    tA[m] = dev_exp2s(s16(counter), exc);
                    counter += 2;
                    if (!mono) {
                        tB[m] = dev_exp2s(s16(counter), exc);
                        counter += 2;
                    }
                }
            }
            for (int m = 0; m < 8; m++) {
                v.samples_A[idx][m] = tA[m];
                v.samples_B[idx][m] = tB[m];
            }
            idx--;
        }
    } else if (it.kind == META_ENTROPY) {
        // `w = new words_data()` with the medians (slow level and bitrate reset)
        for (int k = 0; k < 3; k++) {
            v.median[0][k] = dev_exp2s(u16(2 * k), exc);
            v.median[1][k] = mono ? 0 : dev_exp2s(u16(6 + 2 * k), exc);
        }
        v.slow_level[0] = v.slow_level[1] = 0;
        v.bitrate_acc[0] = v.bitrate_acc[1] = 0;
        v.bitrate_delta[0] = v.bitrate_delta[1] = 0;
    } else if (it.kind == META_HYBRID) {
        int bc = 0;
        if ((uint32_t)it.arg & wvf::HYBRID_BITRATE) {
            v.slow_level[0] = dev_exp2s(u16(bc), exc);
            bc += 2;
            if (!mono) {
                v.slow_level[1] = dev_exp2s(u16(bc), exc);
                bc += 2;
            }
        }
        v.bitrate_acc[0] = (int64_t)wvf::shl32(u16(bc), 16);
        bc += 2;
        if (!mono) {
            v.bitrate_acc[1] = (int64_t)wvf::shl32(u16(bc), 16);
            bc += 2;
        }
        if (bc < (int)it.len) {
            v.bitrate_delta[0] = dev_exp2s(s16(bc), exc);
            bc += 2;
            if (!mono) v.bitrate_delta[1] = dev_exp2s(s16(bc), exc);
        } else {
            v.bitrate_delta[0] = v.bitrate_delta[1] = 0;
        }
    }
}

// Bytes one read_decorr_samples iteration consumes for the quirk term
// (0: the C# loop never advances and throws once the passes run out).
WVF_HD int meta_samples_step(int term, bool mono) {
    if (term > wvf::MAX_TERM) return mono ? 4 : 8;
    if (term < 0) return 4;
    return mono ? 2 * term : 4 * term;
}

}  // namespace wvg
