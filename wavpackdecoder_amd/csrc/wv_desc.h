// wv_desc.h -- the host->device block descriptor.
//
// One descriptor per decoded WavPack block: everything unpack_init
// (UnpackUtils.cs:24-68) and the metadata readers leave in the WavpackStream
// before WavpackUnpackSamples starts decoding the block, flattened so a lane
// or wave can load it with a few wide loads.  Built by wv_framing.cpp,
// consumed by wv_decode.hip.
#pragma once
#include <stdint.h>

namespace wvg {

enum BlockKind : uint32_t {
    KIND_PCM = 0,        // UnpackUtils.unpack_samples path
    KIND_DSD_RAW = 1,    // DsdUtils mode 0
    KIND_DSD_FAST = 2,   // DsdUtils mode 1 (decode_fast)
    KIND_DSD_HIGH = 3,   // DsdUtils mode 3 (decode_high)
    KIND_SKIP = 4,       // nothing to decode on the device (error already known)
};

// status bits written per block by the kernels (and by the framing for
// blocks it already knows the verdict of)
enum StatusBits : uint32_t {
    ST_CRC_CHECKED = 1u << 0,  // the block ran to its end: check_crc_error applies
    ST_CRC_ERROR = 1u << 1,    // check_crc_error() was true (WavPackUtils.cs:273-275)
    ST_MUTED = 1u << 2,        // mute_error was raised in some chunk
    ST_BITS_ERROR = 1u << 3,   // get_words hit the 33-ones / 17-ones break
    ST_EXCEPTION = 1u << 4,    // the reference would raise a C# exception here
    ST_UNSUPPORTED = 1u << 5,  // a layout the device does not decode (malformed files only; wv_framing.cpp)
    ST_DSD_MUTE = 1u << 6,     // DSD chunk(s) muted with 0x55 (post-pass fill, DsdUtils.cs:104-117)
    ST_NONDET = 1u << 7,       // reference output depends on stale caller-buffer contents
    ST_TIMEOUT = 1u << 8,      // a kernel's bounded LDS wait ran out (decoder fault, not a reference outcome)
    ST_REDONE = 1u << 9,       // handed back by the lane kernel and decoded by its fallback (block status only)
};

constexpr int MAXP = 16;  // MAX_NTERMS
constexpr uint32_t kLaneGap = 0xFFFFFFFFu;  // an empty lane in a lane kernel's block list

struct alignas(16) BlockDesc {
    // --- bitstreams (byte offsets into the batch blob)
    uint64_t bits_off;      // ID_WV_BITSTREAM payload (PCM) or DSD payload start (after mult/mode bytes)
    uint64_t out_off;       // int32 index of the block's first output value
    uint64_t wvx_off;       // ID_WVX payload (after the 4 crc bytes), if any
    uint32_t bits_len;      // payload bytes that are real (past them everything reads 0xFF)
    uint32_t wvx_len;       // bytes of the wvx stream counted from wvx_off (end - 4)
    uint32_t kind;          // BlockKind
    uint32_t flags;         // header flags
    uint32_t nframes;       // frames this block decodes (<= block_samples)
    uint32_t block_samples; // header block_samples (CRC is checked only when nframes reaches it)
    int32_t crc;            // expected header crc
    int32_t crc_mvx;        // expected wvx crc
    uint32_t first_chunk;   // frames in the first unpack_samples call for this block
    uint32_t chunk;         // frames per later call (the caller's buffer, 4096 for WvDemo)
    uint32_t first_bsp;     // bufferStartPos (ints) of the first call
    uint32_t out_nch;       // ints per output frame (reduced/num channels)
    uint32_t call_nch;      // DSD mute-fill width per frame
    int32_t mute_limit;     // ((1 << MAG) + 2), doubled for hybrid, C# int wrap applied
    // --- fixup (UnpackUtils.cs:1251-1404, FloatUtils.cs:32-56)
    int32_t shift;          // header SHIFT
    int32_t float_shift;    // float_max_exp - float_norm_exp + float_shift (unclamped)
    int32_t int32_sent_bits, int32_zeros, int32_ones, int32_dups, int32_max_width;
    int32_t wvx_state;      // 0: wvxbits == null; bit0 valid, bits1-7 skip bits, bit8 fixup reads it (INT32)
    // --- entropy state (words_data, WordsUtils.cs:75-187)
    int32_t median[2][3];
    int32_t slow_level[2];
    int64_t bitrate_acc[2];
    int64_t bitrate_delta[2];
    // --- decorrelation passes in decoder order (UnpackUtils.cs:156-360)
    int32_t num_terms;
    uint32_t fstatus;       // StatusBits the framing already knows (UNSUPPORTED, NONDET, ...)
    // --- seek (WavPackUtils.cs:521-594): after SetSample the block is decoded from
    // its start by discard calls of pre_chunk frames up to frame pre_end, whose
    // output is dropped; frame pre_end lands at out_off (which then lies
    // pre_end * out_nch ints before the file's output, as a wrapped offset)
    uint32_t pre_end;       // 0: no discard phase
    uint32_t pre_chunk;     // SAMPLE_BUFFER_SIZE / reduced channels (WavPackUtils.cs:576)
    // --- sticky state (UnpackUtils.cs:24-68, Appendix B-8): what this block takes
    // from the decode of the block before it instead of from its own metadata
    uint32_t inherit;         // InheritBits (0: everything comes from the descriptor)
    uint32_t inherit_passes;  // bit i: pass i's weights, bit 16 + i: its samples continue
    uint32_t chain_len;       // first block of a chain: blocks decoded in sequence from it (>= 2)
    uint32_t wvc_len;         // .wvc correction stream bytes (below; 0: the reference's decode)
    // --- exact float output (OPEN_EXACT_FLOAT, beyond the reference): 0 = the
    // reference's float_values; else XF_ON | float_flags | float_max_exp << 8 |
    // ID_FLOAT_INFO's float_shift << 16 (the wvx stream, if any, in wvx_off/len)
    uint32_t xfloat;
    // (everything up to here and term[] is the descriptor's head: the fields the host
    // reads to route a block -- term_set_of, commit_file -- all lie inside the part of
    // a device-framed descriptor the host sees, wv_api.cpp kDescHead)
    int8_t term[MAXP];
    int8_t delta[MAXP];
    int16_t weight_A[MAXP];
    int16_t weight_B[MAXP];
    int32_t samples_A[MAXP][8];
    int32_t samples_B[MAXP][8];
    // --- DSD (DsdUtils.cs:17-54, 149-242, 343-389)
    uint32_t dsd_data_len;  // bytes from bits_off to the end of the sub-block (C# data.Length - byteptr)
    int32_t dsd_history_bins;
    uint64_t dsd_table_off; // offset into the batch's DSD table area (fast mode)
    int32_t dsd_rate_i;
    int32_t dsd_filters[2][7];  // filter1..5, factor (high mode), per channel
    // --- .wvc correction (beyond the reference): the hybrid block's
    // ID_WVC_BITSTREAM in the correction file (wvc_len bytes); crc then holds the .wvc
    // header's crc (of the exact output) and crc_lossy the .wv header's
    uint64_t wvc_off;
    int32_t crc_lossy;
    // --- DSD mode 1 (DsdUtils.cs:149-242): the probability data after the
    // history-bits and max_probability bytes (run-length coded unless
    // max_probability is 0xFF), from which the decode kernel builds its
    // cumulative tables in LDS; bits_off is the first of the 4 value bytes
    int32_t dsd_max_prob;
    uint64_t dsd_prob_off;
};
constexpr uint32_t XF_ON = 1u << 31;

// A block that starts from state an earlier decode left behind: a block without
// one of the metadata sub-blocks that reset it, or one read without unpack_init
// (a header whose block_index is ahead of the stream: WavPackUtils.cs:219-251).
// The framing groups it with the blocks before it, back to one whose state is
// all known, into a chain that one wave decodes in order (decode_chain,
// wv_decode.hip).
enum InheritBits : uint32_t {
    INH_BITS = 1u << 0,     // main bitstream: no ID_WV_BITSTREAM since the last decode
    INH_WVX = 1u << 1,      // wvx bitstream continues
    INH_ENTROPY = 1u << 2,  // words_data continues (no ID_ENTROPY_VARS), except the fields below left clear
    INH_SLOW0 = 1u << 3,    // ... slow_level / bitrate_acc / bitrate_delta per channel: continues
    INH_SLOW1 = 1u << 4,    //     (clear: a hybrid profile re-sent it; the descriptor holds it)
    INH_ACC0 = 1u << 5,
    INH_ACC1 = 1u << 6,
    INH_DLT0 = 1u << 7,
    INH_DLT1 = 1u << 8,
    INH_NOINIT = 1u << 9,   // no unpack_init since the last decode: crc, crc_x, mute_error, bit register continue
    INH_DSD = 1u << 10,     // DSD: no ID_DSD_BLOCK since the last decode -- its data, coder and filters continue
    INH_MEMBER = 1u << 31,  // decoded by the chain kernel after its predecessor
};
static_assert(sizeof(BlockDesc) % 16 == 0, "BlockDesc is loaded with 16-B alignment");

// frames in the call that starts at block frame `start` (the caller's chunk
// schedule seen from inside one block, discard calls of a seek included)
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t next_call_len(const BlockDesc &d, uint32_t start) {
    return start < d.pre_end ? (d.pre_end - start < d.pre_chunk ? d.pre_end - start : d.pre_chunk) : d.chunk;
}

// One piece (<= 64K values) of one file's int32 output for the format
// epilogue (WavpackFormatSamples, WavPackUtils.cs:288-341).
struct FormatSeg {
    uint64_t in_off;   // first int32 of the piece in the batch output
    uint64_t out_off;  // its first byte in the batch PCM image
    uint32_t n;        // values
    uint32_t bps;      // bytes per sample of the file (WavpackGetBytesPerSample)
};

// An output range the reference zero-fills itself: a gap between the frames already
// returned and the next block's first frame (WavPackUtils.cs:227-251).  The framing
// records it (FramingOutput::zeros) and every decode writes it (wv_zero_fill), so a
// decode's output never depends on the buffer's earlier contents.
struct ZeroSeg {
    uint64_t off;  // first int
    uint64_t n;    // ints
};

}  // namespace wvg
