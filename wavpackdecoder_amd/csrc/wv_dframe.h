// wv_dframe.h -- device-side framing: the header walk and the
// sub-block walk that turn a .wv file's bytes into block descriptors, written
// once for the host and the device (WVF_HD) so the CPU suite checks exactly the
// code the kernels run (tests/emu) against the host framing (wv_framing.cpp).
//
// Two passes over a batch of files already resident in the device blob:
//   dframe_walk   one lane per file: WavpackOpenFileInput (WavPackUtils.cs:36-120)
//                 on the first block, then read_next_header (:600-671) block
//                 after block, recording each header's offset;
//   dframe_block  one lane per block: unpack_init's sub-block walk
//                 (UnpackUtils.cs:24-68, MetadataUtils.cs:15-192) and the
//                 descriptor the host framing would snapshot for it, with the
//                 metadata values read by meta_apply (wv_meta.h) and the chunk
//                 schedule of a caller asking for `chunk` frames per call
//                 (WavPackUtils.cs:200-282, WvDemo.cs:110-135).
//
// Scope: the files the reference decodes block after block with every block
// carrying its own state ("regular" files -- what WavPack writes):
//   * headers back to back from byte 0 to the file's end, every one passing
//     read_next_header's test where the previous block ends, block_index
//     running from 0 without gaps, total_samples known and equal to the sum;
//   * every block PCM, or every block DSD mode 0 (raw bytes) or 3 (the high
//     coder: rate and filter bytes; mode 1's tables are built on the host),
//     mono or stereo as the file opened, INITIAL_BLOCK
//     set, block_samples > 0, and its unpack_init succeeds with the decorr
//     terms, entropy variables and bitstream (or ID_DSD_BLOCK) re-sent (no
//     sticky state, B-8),
//     every deferred read inside its sub-block (wv_meta.h's conditions), no
//     wvx/wvc stream, INT32_INFO / FLOAT_INFO / CHANNEL_INFO the same way in
//     every block.
// Any other file is reported `regular = 0` and framed by the host
// (wv_framing.cpp), which restates every other branch; a batch mixes both.
#pragma once
#include <stdint.h>

#include "wv_desc.h"
#include "wv_format.h"
#include "wv_meta.h"

namespace wvg {

// one file of a device-framed batch
struct DFile {
    // in (host)
    uint64_t base;       // first byte in the blob
    uint64_t len;        // bytes
    uint64_t slot;       // first of the file's header-offset slots (len / 32 + 1 of them)
    uint64_t out_base;   // int32 index of the file's output (set between the passes)
    uint32_t first_desc; // descriptor index of its first block (set between the passes)
    uint32_t chunk;      // frames per caller request
    // out (dframe_walk)
    int32_t regular;     // 1: framed on the device; 0: the host frames it
    uint32_t why;        // first reason it is not (DF_*), for diagnostics
    uint32_t nblocks;
    int32_t num_channels, bits_per_sample, bytes_per_sample, version, mode, is_float, nch;
    // the parallel header walk of a large file (wv_dframe.hip: scan + rank) before
    // dframe_walk: 1 the slots and nblocks are filled and every header checked,
    // -1 the file is not regular (why set), 0 not ranked (dframe_walk walks it)
    int32_t ranked;
    uint32_t tile0, ntiles;  // the file's tiles in the candidate scan
    uint32_t pad_;
    int64_t sample_rate, total_samples, config_flags;
};

// one block's contributions to its file's FileInfo, reduced on the host
struct DBlock {
    int32_t regular;      // the sub-block walk stayed inside the device scope
    uint32_t why;
    int32_t lossy;        // unpack_init set lossy_blocks (UnpackUtils.cs:56-66)
    int32_t five;         // `five` was set by one of its sub-blocks
    int32_t file_format;  // ID_NEW_CONFIG_BLOCK's value, -1 none
    int32_t info_mask;    // bit 0 INT32_INFO, bit 1 FLOAT_INFO seen
    int32_t num_channels; // ID_CHANNEL_INFO's count, -1 none
    int32_t dsd_mult_log2;  // ID_DSD_BLOCK's rate multiplier (log2), -1 none
    int64_t header_off, header_len, trailer_off, trailer_len;  // file-relative, -1 none
};

enum DFrameWhy : uint32_t {
    DF_OK = 0,
    DF_HEADER = 1,      // no valid header where one must start
    DF_OPEN = 2,        // the first block does not open as a plain file
    DF_WALK = 3,        // block_index gap, block_samples 0, layout change, trailing bytes
    DF_TOTAL = 4,       // total_samples unknown or not the sum of the blocks
    DF_SUBBLOCK = 5,    // sub-block walk fails or runs past the block
    DF_STATE = 6,       // a block continues state (no terms / entropy / bitstream re-sent)
    DF_KIND = 7,        // DSD, wvx, wvc, an unsupported layout
    DF_READER = 8,      // a reader the host runs itself (reads past its sub-block, or fails)
    DF_UNIFORM = 9,     // INT32/FLOAT/CHANNEL info not the same way in every block
    DF_SLOTS = 10,      // more blocks than slots
};

// the header fields one block's walk needs (WavpackHeader.cs:15-22)
struct DHdr {
    uint32_t ckSize, block_samples, flags;
    int32_t crc;
    int16_t version;
    int64_t total_samples, block_index;
};

// read_next_header's acceptance test and field decode at exactly `pos`
// (WavPackUtils.cs:600-671 without the resync scan)
WVF_HD bool dframe_header(const uint8_t *f, uint64_t len, uint64_t pos, DHdr &h) {
    if (pos + 32 > len) return false;
    const uint8_t *b = f + pos;
    if (!(b[0] == 'w' && b[1] == 'v' && b[2] == 'p' && b[3] == 'k' && (b[4] & 1) == 0 && b[6] < 16 && b[7] == 0 &&
          b[9] == 4 && b[8] >= (wvf::MIN_STREAM_VERS & 0xff) && b[8] <= (wvf::MAX_STREAM_VERS & 0xff)))
        return false;
    h.ckSize = (uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24);
    h.version = (int16_t)((b[9] << 8) | b[8]);
    h.total_samples = (int64_t)(((uint64_t)b[11] << 32) | ((uint64_t)b[15] << 24) | ((uint64_t)b[14] << 16) |
                                ((uint64_t)b[13] << 8) | b[12]);
    h.block_index = (int64_t)(((uint64_t)b[10] << 32) | ((uint64_t)b[19] << 24) | ((uint64_t)b[18] << 16) |
                              ((uint64_t)b[17] << 8) | b[16]);
    h.block_samples = (uint32_t)b[20] | ((uint32_t)b[21] << 8) | ((uint32_t)b[22] << 16) | ((uint32_t)b[23] << 24);
    h.flags = (uint32_t)b[24] | ((uint32_t)b[25] << 8) | ((uint32_t)b[26] << 16) | ((uint32_t)b[27] << 24);
    h.crc = (int32_t)((uint32_t)b[28] | ((uint32_t)b[29] << 8) | ((uint32_t)b[30] << 16) | ((uint32_t)b[31] << 24));
    return true;
}

// what one block's unpack_init leaves in the stream and the context (the
// fields a regular block sets), plus the file-level values it touches
struct DState {
    int32_t num_terms;
    int8_t term[wvf::MAX_NTERMS], delta[wvf::MAX_NTERMS];
    MetaItem items[6];  // deferred reads in stream order (file offsets)
    int32_t nitems;
    int64_t bits_off;   // ID_WV_BITSTREAM data, file offset
    int32_t bits_len;
    int32_t i32[4];     // sent_bits, zeros, ones, dups
    int32_t fl[4];      // float flags, shift, max_exp, norm_exp
    bool terms, entropy, bits, has_i32, has_fl;
    // ID_DSD_BLOCK, modes 0 and 3 (DsdUtils.cs:17-54, 343-389): the payload after
    // mult/mode (and mode 3's rate and filter bytes)
    bool dsd;
    int32_t dsd_mode;
    int32_t dsd_mult_log2;  // data[0] & 31
    int64_t dsd_off;        // file offset of the payload (data[byteptr])
    int32_t dsd_len;        // C# data.Length - byteptr
    int32_t dsd_rate_i;     // mode 3: init_ptable's rate index
    int32_t dsd_filt[2][6]; // mode 3: filter1..5 << 12, factor
    int32_t dsd_bins;       // mode 1: history bins
    int32_t dsd_maxp;       // mode 1: max_probability
    int64_t dsd_prob;       // mode 1: file offset of the probability data
    // context (file-level) values, updated in place
    int64_t cfg_flags;
    int32_t xmode;
    int32_t num_channels;   // -1: no ID_CHANNEL_INFO in this block
    int64_t sample_rate;    // -1: none
    bool five;
    int32_t file_format;    // -1: none
    int64_t header_off, header_len, trailer_off, trailer_len;
};

WVF_HD void dstate_init(DState &s) {
    s.num_terms = 0;
    for (int i = 0; i < wvf::MAX_NTERMS; i++) s.term[i] = s.delta[i] = 0;
    s.nitems = 0;
    s.bits_off = 0;
    s.bits_len = 0;
    for (int i = 0; i < 4; i++) s.i32[i] = s.fl[i] = 0;
    s.terms = s.entropy = s.bits = s.has_i32 = s.has_fl = false;
    s.dsd = false;
    s.dsd_mode = 0;
    s.dsd_mult_log2 = 0;
    s.dsd_off = 0;
    s.dsd_len = 0;
    s.dsd_rate_i = 0;
    s.dsd_bins = s.dsd_maxp = 0;
    s.dsd_prob = 0;
    for (int c = 0; c < 2; c++)
        for (int k = 0; k < 6; k++) s.dsd_filt[c][k] = 0;
    s.cfg_flags = 0;
    s.xmode = 0;
    s.num_channels = -1;
    s.sample_rate = -1;
    s.five = false;
    s.file_format = -1;
    s.header_off = s.header_len = s.trailer_off = s.trailer_len = -1;
}

// drop pending reads a later read overwrites completely (wv_framing.cpp drop_pending)
WVF_HD void dstate_drop(DState &s, uint32_t k0, uint32_t k1) {
    int o = 0;
    for (int i = 0; i < s.nitems; i++)
        if (s.items[i].kind != k0 && s.items[i].kind != k1) s.items[o++] = s.items[i];
    s.nitems = o;
}

WVF_HD bool dstate_push(DState &s, uint64_t off, uint32_t kind, int32_t len, int32_t arg, int32_t counter0, bool mono) {
    if (s.nitems >= 6) return false;
    MetaItem &it = s.items[s.nitems++];
    it.off = off;
    it.kind = kind;
    it.len = (uint32_t)len;
    it.num_terms = s.num_terms;
    it.arg = arg;
    it.counter0 = counter0;
    it.mono = mono ? 1u : 0u;
    return true;
}

// unpack_init's sub-block walk over the block whose header is at `hpos`
// (read_metadata_buff MetadataUtils.cs:15-109, process_metadata :111-192, the
// readers of UnpackUtils.cs:156-491 / WordsUtils.cs:75-187 / FloatUtils.cs:15-30);
// DF_OK when the block stays inside the device scope
WVF_HD uint32_t dframe_subblocks(const uint8_t *f, uint64_t len, uint64_t hpos, const DHdr &h, DState &s) {
    using namespace wvf;
    const bool mono = (h.flags & MONO_DATA) != 0;
    uint64_t pos = hpos + 32;
    int64_t bytecount = 24;
    while (bytecount < (int64_t)h.ckSize) {
        if (pos + 2 > len) return DF_SUBBLOCK;
        uint8_t id = f[pos];
        int t = f[pos + 1];
        pos += 2;
        bytecount += 2;
        int32_t byte_length = t << 1;
        if (id & ID_LARGE) {
            id &= (uint8_t)~ID_LARGE;
            if (pos + 2 > len) return DF_SUBBLOCK;
            byte_length += (int32_t)f[pos] << 9;
            byte_length += (int32_t)f[pos + 1] << 17;
            pos += 2;
            bytecount += 2;
        }
        const int32_t to_read = byte_length;
        if (id & ID_ODD_SIZE) {
            id &= (uint8_t)~ID_ODD_SIZE;
            byte_length--;
        }
        if (byte_length < 0) return DF_SUBBLOCK;
        const bool hasdata = byte_length > 0;
        const uint64_t doff = pos;
        if (hasdata) {
            bytecount += to_read;
            if (pos + (uint64_t)to_read > len) return DF_SUBBLOCK;  // a short read fails the block
            pos += (uint64_t)to_read;
        }
        const uint8_t *d = f + doff;
        switch (id) {
        case ID_DUMMY:
        case ID_SHAPING_WEIGHTS: break;
        case ID_DECORR_TERMS: {  // UnpackUtils.cs:156-187
            if (byte_length > MAX_NTERMS) return DF_READER;
            for (int c = 0; c < byte_length; c++) {
                const int dc = byte_length - 1 - c;
                const int term = (d[c] & 0x1f) - 5;
                if (term < -3 || (term > MAX_TERM && term < 17) || term > 18) return DF_READER;
                s.term[dc] = (int8_t)term;
                s.delta[dc] = (int8_t)((d[c] >> 5) & 7);
            }
            for (int i = byte_length; i < MAX_NTERMS; i++) s.term[i] = s.delta[i] = 0;
            s.num_terms = byte_length;
            s.terms = true;
            dstate_drop(s, META_WEIGHTS, META_SAMPLES);
            break;
        }
        case ID_DECORR_WEIGHTS: {  // UnpackUtils.cs:196-239
            if (!s.terms) return DF_STATE;
            const int termcnt = mono ? byte_length : byte_length / 2;
            if (termcnt > s.num_terms) return DF_READER;
            if (termcnt > 0 && !dstate_push(s, doff, META_WEIGHTS, byte_length, termcnt, 0, mono)) return DF_READER;
            break;
        }
        case ID_DECORR_SAMPLES: {  // UnpackUtils.cs:250-360 (quirk B-7 in meta_apply)
            if (!s.terms) return DF_STATE;
            const int q = s.num_terms > 0 ? s.term[s.num_terms - 1] : 0;
            const int c0 = (h.version == 0x402 && (h.flags & HYBRID_FLAG)) ? (mono ? 2 : 4) : 0;
            const int step = meta_samples_step(q, mono), span = byte_length - c0;
            if (!(span <= 0 || (step > 0 && span % step == 0 && span / step <= s.num_terms))) return DF_READER;
            if (s.num_terms > 0 && !dstate_push(s, doff, META_SAMPLES, byte_length, q, c0, mono)) return DF_READER;
            break;
        }
        case ID_ENTROPY_VARS:  // WordsUtils.cs:75-116
            if (!(mono ? byte_length >= 6 : byte_length == 12)) return DF_READER;
            dstate_drop(s, META_ENTROPY, META_HYBRID);
            if (!dstate_push(s, doff, META_ENTROPY, byte_length, 0, 0, mono)) return DF_READER;
            s.entropy = true;
            break;
        case ID_HYBRID_PROFILE: {  // WordsUtils.cs:124-187
            const int w2 = mono ? 2 : 4;
            int need = ((h.flags & HYBRID_BITRATE) ? w2 : 0) + w2;
            if (need < byte_length) need += w2;
            if (need != byte_length) return DF_READER;
            if (!dstate_push(s, doff, META_HYBRID, byte_length, (int32_t)h.flags, 0, mono)) return DF_READER;
            break;
        }
        case ID_FLOAT_INFO:  // FloatUtils.cs:15-30
            if (byte_length != 4) return DF_READER;
            for (int i = 0; i < 4; i++) s.fl[i] = d[i];
            s.has_fl = true;
            break;
        case ID_INT32_INFO:  // UnpackUtils.cs:367-382
            if (byte_length != 4) return DF_READER;
            for (int i = 0; i < 4; i++) s.i32[i] = d[i];
            s.has_i32 = true;
            break;
        case ID_CHANNEL_INFO:  // UnpackUtils.cs:389-410 (the mask is not on the path)
            if (byte_length == 0 || byte_length > 5) return DF_READER;
            s.num_channels = d[0];
            break;
        case ID_CONFIG_BLOCK: {  // UnpackUtils.cs:432-455
            int bytecnt = byte_length, counter = 0;
            if (bytecnt >= 3) {
                s.cfg_flags &= 0xff;
                s.cfg_flags |= (int64_t)shl32(d[counter++], 8);
                s.cfg_flags |= (int64_t)shl32(d[counter++], 16);
                s.cfg_flags |= (int64_t)shl32(d[counter++], 24);
            }
            if (bytecnt >= 4 && (s.cfg_flags & CONFIG_EXTRA_MODE)) {
                s.xmode = d[counter++];
                bytecnt--;
            }
            if (bytecnt >= 5) s.five = true;
            break;
        }
        case ID_SAMPLE_RATE:  // UnpackUtils.cs:459-473
            if (byte_length == 3) s.sample_rate = (int64_t)d[0] | (int64_t)shl32(d[1], 8) | (int64_t)shl32(d[2], 16);
            break;
        case ID_WV_BITSTREAM:  // UnpackUtils.cs:75-90 (copy_data fails on an empty sub-block)
            if (!hasdata) return DF_READER;
            s.bits = true;
            s.bits_off = (int64_t)doff;
            s.bits_len = byte_length;
            break;
        case ID_NEW_CONFIG_BLOCK:
            s.five = true;
            if (byte_length >= 1) s.file_format = d[0];
            break;
        case ID_RIFF_HEADER:
        case ID_ALT_HEADER:  // UnpackUtils.cs:475-491
            s.header_off = (int64_t)doff;
            s.header_len = byte_length;
            break;
        case ID_RIFF_TRAILER:
        case ID_ALT_TRAILER:
            s.trailer_off = (int64_t)doff;
            s.trailer_len = byte_length;
            break;
        case ID_ALT_EXTENSION: break;
        case ID_BLOCK_CHECKSUM: s.five = true; break;
        case ID_WVC_BITSTREAM:
        case ID_WVX_BITSTREAM:
        case ID_WVX_NEW_BITSTREAM: return DF_KIND;  // a second stream: the host frames the file
        case ID_DSD_BLOCK: {  // init_dsd_block (DsdUtils.cs:17-54)
            if (byte_length < 2 || d[0] > 31 || (d[1] != 0 && d[1] != 1 && d[1] != 3)) return DF_KIND;
            // copy_data's length: the read buffer's fill for a small sub-block, the bytes read for a large one
            const int32_t dl = to_read > BITSTREAM_BUFFER_SIZE ? to_read : byte_length;
            int32_t p = 2;
            if (d[1] == 0) {
                if ((int64_t)(dl - 2) != (int64_t)h.block_samples * (mono ? 1 : 2)) return DF_READER;
            } else if (d[1] == 1) {
                // init_dsd_block_fast (:149-242), its checks only: the decode kernel builds the
                // cumulative tables from the probability data itself
                if (p == dl) return DF_READER;
                const int hbits = d[p++];
                if (p == dl || hbits > 5) return DF_READER;
                const int bins = 1 << hbits, outend = bins * 256;
                const int maxp = d[p++];
                s.dsd_bins = bins;
                s.dsd_maxp = maxp;
                s.dsd_prob = (int64_t)doff + p;
                // the per-bin sums are ushort (wrapping); bins fill in order, so one running sum
                int total = 0, cur = 0;
                uint32_t sum = 0;
                if (maxp < 0xFF) {
                    int outptr = 0;
                    while (outptr < outend && p < dl) {
                        const int code = d[p++];
                        if (code > maxp) {
                            const int z = code - maxp;
                            outptr += z < outend - outptr ? z : outend - outptr;
                        } else if (code != 0) {
                            if ((outptr >> 8) != cur) {
                                total += (int)(sum & 0xFFFFu);
                                sum = 0;
                                cur = outptr >> 8;
                            }
                            sum += (uint32_t)code;
                            outptr++;
                        } else {
                            break;
                        }
                    }
                    if (outptr < outend || (p < dl && d[p++] > 0)) return DF_READER;
                } else if (dl - p > outend) {
                    for (int i = 0; i < outend; i++) {
                        if ((i >> 8) != cur) {
                            total += (int)(sum & 0xFFFFu);
                            sum = 0;
                            cur = i >> 8;
                        }
                        sum += d[p + i];
                    }
                    p += outend;
                } else {
                    return DF_READER;
                }
                total += (int)(sum & 0xFFFFu);
                if (dl - p < 4 || total > bins * 1280) return DF_READER;
            } else {  // init_dsd_block_high (:343-389); its ptable is built by the decode kernel
                if (dl - 2 < (mono ? 13 : 20) || d[3] != 20) return DF_READER;
                s.dsd_rate_i = d[2];
                p = 4;
                for (int c = 0; c < (mono ? 1 : 2); c++) {
                    for (int k = 0; k < 5; k++) s.dsd_filt[c][k] = (int32_t)d[p++] << 12;
                    const uint32_t fv = (uint32_t)d[p] | ((uint32_t)d[p + 1] << 8);
                    p += 2;
                    s.dsd_filt[c][5] = (int32_t)(fv << 16) >> 16;
                }
            }
            s.dsd = true;
            s.dsd_mode = d[1];
            s.dsd_mult_log2 = d[0] & 31;
            s.dsd_off = (int64_t)doff + p;
            s.dsd_len = dl - p;
            break;
        }
        default:
            if (!(id & ID_OPTIONAL_DATA)) return DF_READER;  // "invalid metadata id": the host reports it
            break;
        }
    }
    if (bytecount != (int64_t)h.ckSize) return DF_SUBBLOCK;
    if (h.flags & DSD_FLAG) return s.dsd ? DF_OK : DF_STATE;  // unpack_init: dsd.ready (a block without
                                                              // ID_DSD_BLOCK continues the consumed DSD state)
    if (!s.bits || s.bits_len == 0) return DF_READER;  // "invalid WavPack file"
    if (!s.terms || !s.entropy) return DF_STATE;       // passes / words_data continue the previous decode
    return DF_OK;
}

// WavpackOpenFileInput on the first block + the header walk, for file fi.
// `slots` receives each block's header offset (file-relative).
WVF_HD void dframe_walk(DFile &fi, const uint8_t *blob, uint64_t *slots) {
    using namespace wvf;
    const uint8_t *f = blob + fi.base;
    const uint64_t len = fi.len, cap = len / 32 + 1;
    fi.regular = 0;
    if (fi.ranked < 0) return;  // the parallel walk found it irregular (why set)
    if (fi.ranked == 0) fi.nblocks = 0;
    DHdr h;
    if (!dframe_header(f, len, 0, h)) {
        fi.why = DF_HEADER;
        return;
    }
    if (h.block_samples == 0 || h.block_index != 0 ||
        ((h.flags & DSD_FLAG) && (h.flags & FALSE_STEREO))) {  // DSD mode 0 + FALSE_STEREO overruns (DsdUtils.cs:81)
        fi.why = DF_OPEN;
        return;
    }
    if (h.total_samples == 0xFFFFFFFFLL) {
        fi.why = DF_TOTAL;
        return;
    }
    DState s;
    dstate_init(s);
    uint32_t why = dframe_subblocks(f, len, 0, h, s);
    if (why != DF_OK) {
        fi.why = why;
        return;
    }
    // open_input (WavPackUtils.cs:36-120) after the first block's unpack_init
    const bool lossy0 = ((h.flags & INT32_DATA) && s.i32[0] != 0) ||
                        ((h.flags & FLOAT_DATA) && (s.fl[0] & (FLOAT_EXCEPTIONS | FLOAT_ZEROS_SENT | FLOAT_SHIFT_SENT |
                                                              FLOAT_SHIFT_SAME)));
    int64_t cfg = (s.cfg_flags & ~0xffLL) | (h.flags & 0xff);
    int bytes_per_sample = (int)((h.flags & BYTES_STORED) + 1);
    int bits_per_sample = (int)(bytes_per_sample * 8 - ((h.flags & SHIFT_MASK) >> SHIFT_LSB));
    if (cfg & FLOAT_DATA) {
        bytes_per_sample = 3;
        bits_per_sample = 24;
    }
    int64_t rate = s.sample_rate >= 0 ? s.sample_rate : 0;
    if (rate == 0) {
        const int64_t rates[15] = {6000,  8000,  9600,  11025, 12000, 16000, 22050, 24000,
                                   32000, 44100, 48000, 64000, 88200, 96000, 192000};
        rate = ((h.flags & SRATE_MASK) == SRATE_MASK) ? 44100 : rates[(h.flags & SRATE_MASK) >> SRATE_LSB];
    }
    int num_channels = s.num_channels > 0 ? s.num_channels : 0;
    if (num_channels == 0) num_channels = (h.flags & MONO_FLAG) ? 1 : 2;
    if (num_channels > 2 || s.num_channels == 0) {  // "only two channels supported!" / a zero count
        fi.why = DF_OPEN;
        return;
    }
    int mode = 0;  // WavpackGetMode (WavPackUtils.cs:133-167) at open
    if (cfg & CONFIG_HYBRID_FLAG) mode |= 0x4;
    else if (!(cfg & CONFIG_LOSSY_MODE)) mode |= 0x2;
    if (lossy0) mode &= ~0x2;
    if (cfg & CONFIG_FLOAT_DATA) mode |= 0x8;
    if (cfg & CONFIG_HIGH_FLAG) {
        mode |= 0x20;
        if ((cfg & CONFIG_VERY_HIGH_FLAG) || h.version < 0x405) mode |= 0x400;
    }
    if (cfg & CONFIG_FAST_FLAG) mode |= 0x40;
    if (cfg & CONFIG_EXTRA_MODE) mode |= 0x80 | ((s.xmode << 12) & 0x7000);
    if (h.flags & DSD_FLAG) {  // dsd_multiplier > 0 (open_input, WavPackUtils.cs:116-119)
        mode |= 0x10000;
        bytes_per_sample = 1;
        bits_per_sample = 8;
    }
    fi.num_channels = num_channels;
    fi.nch = num_channels;
    fi.bits_per_sample = bits_per_sample;
    fi.bytes_per_sample = bytes_per_sample;
    fi.version = h.version;
    fi.mode = mode;
    fi.is_float = (cfg & CONFIG_FLOAT_DATA) != 0;
    fi.sample_rate = rate;
    fi.total_samples = h.total_samples;
    fi.config_flags = cfg;
    // the header walk: every block starts where the previous one ends
    const uint32_t bch0 = (uint32_t)num_channels;
    const uint32_t h0flags = h.flags;
    if (fi.ranked == 1) {  // walked in parallel: every header checked but against block 0's layout
        if (((h.flags & MONO_FLAG) ? 1u : 2u) != bch0) {
            fi.why = DF_WALK;
            return;
        }
        fi.why = DF_OK;
        fi.regular = 1;
        return;
    }
    uint64_t pos = 0;
    int64_t sum = 0;
    uint32_t n = 0;
    for (;;) {
        const uint32_t bch = (h.flags & MONO_FLAG) ? 1u : 2u;
        if (h.block_samples == 0 || !(h.flags & INITIAL_BLOCK) || h.block_index != sum || bch != bch0 ||
            ((h.flags ^ h0flags) & DSD_FLAG) || ((h.flags & DSD_FLAG) && (h.flags & FALSE_STEREO)) ||
            ((h.flags & FALSE_STEREO) && (h.flags & MONO_FLAG))) {
            fi.why = DF_WALK;
            return;
        }
        if (n >= cap) {
            fi.why = DF_SLOTS;
            return;
        }
        slots[fi.slot + n++] = pos;
        sum += h.block_samples;
        pos += (uint64_t)h.ckSize + 8;
        if (sum > fi.total_samples) {
            fi.why = DF_TOTAL;
            return;
        }
        if (pos == len) break;
        if (sum == fi.total_samples || !dframe_header(f, len, pos, h)) {
            fi.why = DF_WALK;
            return;
        }
    }
    if (sum != fi.total_samples) {
        fi.why = DF_TOTAL;
        return;
    }
    fi.nblocks = n;
    fi.why = DF_OK;
    fi.regular = 1;
}

// one block of a regular file: its descriptor (the host framing's snapshot,
// with the deferred values applied) and its FileInfo contributions
WVF_HD void dframe_block(const DFile &fi, uint32_t k, const uint8_t *blob, const uint64_t *slots, BlockDesc &d,
                         DBlock &r) {
    using namespace wvf;
    const uint8_t *f = blob + fi.base;
    const uint64_t hpos = slots[fi.slot + k];
    {  // the host's memset (padding included)
        uint32_t *w = reinterpret_cast<uint32_t *>(&d);
        for (uint32_t i = 0; i < sizeof(BlockDesc) / 4; i++) w[i] = 0;
    }
    r.regular = 0;
    r.lossy = r.five = 0;
    r.file_format = -1;
    r.info_mask = 0;
    r.num_channels = -1;
    r.dsd_mult_log2 = -1;
    r.header_off = r.header_len = r.trailer_off = r.trailer_len = -1;
    DHdr h;
    if (!dframe_header(f, fi.len, hpos, h)) {
        r.why = DF_HEADER;
        d.kind = KIND_SKIP;
        return;
    }
    DState s;
    dstate_init(s);
    r.why = dframe_subblocks(f, fi.len, hpos, h, s);
    if (r.why != DF_OK) {
        d.kind = KIND_SKIP;
        return;
    }
    if (s.i32[0] > 32) {  // the host marks it unsupported (wv_framing.cpp snapshot)
        r.why = DF_KIND;
        d.kind = KIND_SKIP;
        return;
    }
    r.regular = 1;
    r.lossy = ((h.flags & INT32_DATA) && s.i32[0] != 0) ||
              ((h.flags & FLOAT_DATA) &&
               (s.fl[0] & (FLOAT_EXCEPTIONS | FLOAT_ZEROS_SENT | FLOAT_SHIFT_SENT | FLOAT_SHIFT_SAME)));
    r.five = s.five;
    r.file_format = s.file_format;
    r.info_mask = (s.has_i32 ? 1 : 0) | (s.has_fl ? 2 : 0);
    r.num_channels = s.num_channels;
    r.dsd_mult_log2 = s.dsd ? s.dsd_mult_log2 : -1;
    r.header_off = s.header_off;
    r.header_len = s.header_len;
    r.trailer_off = s.trailer_off;
    r.trailer_len = s.trailer_len;
    // snapshot (wv_framing.cpp Framer::snapshot)
    const uint32_t flags = h.flags;
    d.flags = flags;
    d.block_samples = h.block_samples;
    d.crc = h.crc;
    const int mag = (int)((flags & MAG_MASK) >> MAG_LSB);
    int32_t ml = (int32_t)((int64_t)(1LL << mag) + 2);
    if (flags & HYBRID_FLAG) ml = mul32(ml, 2);
    d.mute_limit = ml;
    d.shift = (int32_t)((flags & SHIFT_MASK) >> SHIFT_LSB);
    d.float_shift = s.fl[2] - s.fl[3] + s.fl[1];
    d.int32_sent_bits = s.i32[0];
    d.int32_zeros = s.i32[1];
    d.int32_ones = s.i32[2];
    d.int32_dups = s.i32[3];
    if (flags & DSD_FLAG) {  // DSD mode 0 (DsdUtils.cs:60-147: the raw bytes) or 3 (:391-493)
        d.kind = s.dsd_mode == 3 ? KIND_DSD_HIGH : (s.dsd_mode == 1 ? KIND_DSD_FAST : KIND_DSD_RAW);
        d.bits_off = fi.base + (uint64_t)s.dsd_off;
        d.dsd_data_len = (uint32_t)s.dsd_len;
        d.dsd_rate_i = s.dsd_rate_i;
        if (s.dsd_mode == 1) {  // no table area: the decode kernel builds its tables (dsd_table_off unused)
            d.dsd_history_bins = s.dsd_bins;
            d.dsd_max_prob = s.dsd_maxp;
            d.dsd_prob_off = fi.base + (uint64_t)s.dsd_prob;
        }
        for (int c = 0; c < 2; c++)
            for (int k = 0; k < 6; k++) d.dsd_filters[c][k] = s.dsd_filt[c][k];
    } else {
        d.kind = KIND_PCM;
        d.bits_off = fi.base + (uint64_t)s.bits_off;
        d.bits_len = (uint32_t)s.bits_len;
        d.num_terms = s.num_terms;
        for (int i = 0; i < s.num_terms; i++) {
            d.term[i] = s.term[i];
            d.delta[i] = s.delta[i];
        }
        for (int i = 0; i < s.nitems; i++) meta_apply(d, s.items[i], f);
    }
    // the caller's chunk schedule: block k starts at file frame block_index
    const uint64_t nch = (uint64_t)fi.nch, chunk = fi.chunk, at = (uint64_t)h.block_index;
    const uint64_t into = at % chunk;
    d.out_off = fi.out_base + at * nch;
    d.first_chunk = (uint32_t)(chunk - into < h.block_samples ? chunk - into : h.block_samples);
    d.chunk = (uint32_t)chunk;
    d.first_bsp = (uint32_t)(into * nch);
    d.out_nch = (uint32_t)nch;
    d.call_nch = (fi.num_channels == 1 || (flags & MONO_FLAG)) ? 1 : 2;
    d.nframes = h.block_samples;
}

}  // namespace wvg
