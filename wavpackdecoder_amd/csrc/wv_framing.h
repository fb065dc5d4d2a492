// wv_framing.h -- host-side framing: .wv file bytes -> device block descriptors.
//
// Restates the part of the reference that runs *around* the hot path:
//   WavpackOpenFileInput   (WavPackUtils.cs:36-120)
//   read_next_header       (WavPackUtils.cs:600-671)
//   unpack_init + readers  (UnpackUtils.cs:24-491, MetadataUtils.cs, WordsUtils.cs:75-187,
//                           FloatUtils.cs:15-30, DsdUtils.cs:17-54,149-242,343-389)
//   the block-walking loop of WavpackUnpackSamples (WavPackUtils.cs:200-282)
//     driven by a caller that asks for `chunk` frames per call (WvDemo.cs:110-135)
// It produces one BlockDesc per decoded block with the exact start state, the
// output offset and the chunk seams.  No sample is decoded here.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "wv_desc.h"
#include "wv_dframe.h"
#include "wv_meta.h"

namespace wvg {

struct FileInfo {
    // WavpackOpenFileInput outcome (WavPackUtils.cs:36-120)
    int32_t open_ok = 0;
    std::string error;  // wpc.error_message (empty when none)
    int32_t num_channels = 0, reduced_channels = 0, bits_per_sample = 0, bytes_per_sample = 0;
    int32_t version = 0, mode = 0, is_float = 0, is_five = 0, file_format = 0;
    int64_t sample_rate = 0, total_samples = -1, config_flags = 0;
    uint32_t dsd_multiplier = 0;
    int32_t lossy_blocks = 0;   // after the whole walk
    int32_t exception = 0;      // framing hit a C# exception; output stops there
    int32_t nondet = 0;
    // output of the chunked caller
    int32_t out_nch = 0;        // ints per frame
    int64_t out_frames = 0;     // frames all calls return
    int64_t first_call_frames = -1;  // frames the first call returns (-1: it threw)
    // output frame counts at which a call returned fewer frames than it asked for (the
    // reference's loop breaks on a header or unpack_init failure, WavPackUtils.cs:215-221;
    // and the file's last call): the stream API ends its calls there too
    std::vector<int64_t> call_cuts;
    int32_t seek_result = 0;    // SetSample: 1 positioned, 0 false, -1 exception (0 when no seek was asked)
    int64_t sample_index0 = 0;  // stream.sample_index when the caller's first (non-discard) call starts
    uint64_t blob_base = 0;     // the file's first byte inside the batch blob (header/trailer offsets are file-relative)
    int64_t header_off = -1, header_len = 0, trailer_off = -1, trailer_len = 0;  // RIFF/ALT header+trailer
    // blocks of this file inside the batch descriptor array
    int64_t first_desc = 0, num_desc = 0;
};

// DSD fast/high tables live in a side area (bytes) appended per block.
struct FramingOutput {
    std::vector<ZeroSeg> zeros;   // gap zero-fills (ZeroSeg)
    std::vector<BlockDesc> descs;
    std::vector<uint8_t> tables;  // DSD tables (see BlockDesc::dsd_table_off)
    // defer_values: the decorr weight/sample and entropy/hybrid values are left
    // to meta_apply (wv_meta.h) -- the device parse kernel, or apply_meta_jobs on
    // the host; until then those descriptor fields hold the older stream values
    bool defer_values = false;
    // chain_tables_only: keep the DSD mode-1 tables only for blocks in a decode chain
    // (the device's decode_dsd_chain reads them; every other mode-1 block has its tables
    // built on the device, dsd_fast_tables / wv_dsd1_lane), so a batch does not copy and
    // upload ~2 KB per history bin of every mode-1 block
    bool chain_tables_only = false;
    std::vector<MetaItem> items;  // offsets into the batch blob
    std::vector<MetaJob> jobs;
};

// Host application of the deferred metadata values (what wv_meta_parse does on
// the device); `blob` is the buffer the item offsets point into.
void apply_meta_jobs(FramingOutput &out, const uint8_t *blob);

// Frame one file.  `file` must stay valid until the batch is uploaded.
// `blob_base` is the file's byte offset inside the device blob; descriptors are
// appended to `out` with out_off relative to `out_base_ints`.
// seek_to >= 0: the caller calls SetSample(seek_to) (WavPackUtils.cs:509-594)
// right after opening, and its calls return the frames from there on.
// wvc (optional): the file's .wvc correction file, whose bytes start at blob
// offset wvc_base; hybrid blocks then decode exactly (beyond the reference).
void frame_file(const uint8_t *file, size_t len, uint64_t blob_base, uint64_t out_base_ints, uint32_t open_flags,
                int chunk, FramingOutput &out, FileInfo &info, int64_t seek_to = -1, const uint8_t *wvc = nullptr,
                size_t wvc_len = 0, uint64_t wvc_base = 0);

// Output ints a batch reserves for a framed file: its reported values
// (out_frames x out_nch) or more when a descriptor writes past them -- a file
// that raised the C# exception mid-call keeps the descriptor of that call,
// whose writes must not reach the next file's range.
int64_t file_out_extent(const FramingOutput &out, const FileInfo &info, uint64_t out_base_ints);

// FileInfo of a file framed on the device (wv_dframe.h) from its walk and its
// blocks' records (nblocks of them); false when a block left the device scope
// or the blocks disagree on what they carry (the host frames the file instead).
// first_desc / blob_base are the caller's.
bool dframe_file_info(const DFile &df, const DBlock *blocks, FileInfo &fi);

// WavpackGetMode (WavPackUtils.cs:133-167) from the framed context values
int compute_mode(const FileInfo &info);

}  // namespace wvg
