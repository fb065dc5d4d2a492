// tests/emu/emu.cpp -- TEST-ONLY host build of the device decode core.
//
// Compiles wv_framing.cpp + wv_decode_core.h (the exact source the HIP kernel
// runs) for the host, so `pytest -m "not gpu"` can check the decode logic
// against the oracle on a machine without a GPU.  It is never loaded by the
// product package (wavpackdecoder_amd), which only runs the HIP kernels.
#include <stddef.h>
#include <string.h>

#include <vector>

#include "../../wavpackdecoder_amd/csrc/wv_decode_core.h"
#include "../../wavpackdecoder_amd/csrc/wv_framing.h"

using namespace wvg;

struct HostStore {
    int32_t *out;
    uint64_t base;  // may be a wrapped negative offset (a seek's discarded frames precede it)
    uint64_t skip;
    void put(uint64_t i, int32_t v) {
        if (i >= skip) out[base + i] = v;
    }
};

extern "C" {
// the descriptor layout the Python side indexes raw descriptor bytes with
int emu_desc_layout(int64_t *out, int n) {
    const int64_t v[7] = {(int64_t)sizeof(BlockDesc), (int64_t)offsetof(BlockDesc, kind),
                          (int64_t)offsetof(BlockDesc, dsd_table_off), (int64_t)offsetof(BlockDesc, inherit),
                          (int64_t)offsetof(BlockDesc, median), (int64_t)offsetof(BlockDesc, bits_off),
                          (int64_t)offsetof(BlockDesc, bits_len)};
    static_assert(offsetof(BlockDesc, chain_len) == offsetof(BlockDesc, inherit) + 8, "inherit, inherit_passes, chain_len");
    for (int i = 0; i < n && i < 7; i++) out[i] = v[i];
    return 7;
}

// Frames n files back to back into one batch the way wvg_batch_add_file does
// and counts descriptor writes outside their file's reserved output range:
// *bad_reserved with file_out_extent (the product rule), *bad_values when only
// the reported values (out_frames x out_nch) were reserved.
void emu_batch_ranges(const uint8_t *blob, const uint64_t *offs, const uint64_t *lens, int n, int chunk,
                      int64_t *bad_reserved, int64_t *bad_values) {
    FramingOutput fo;
    fo.defer_values = true;
    *bad_reserved = *bad_values = 0;
    int64_t base = 0;
    for (int i = 0; i < n; i++) {
        FileInfo fi;
        frame_file(blob + offs[i], (size_t)lens[i], offs[i], (uint64_t)base, 0, chunk, fo, fi);
        if (!fi.open_ok) continue;
        const int64_t ext = file_out_extent(fo, fi, (uint64_t)base);
        const int64_t vals = fi.out_frames * fi.out_nch;
        for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++) {
            const BlockDesc &d = fo.descs[(size_t)k];
            if (d.kind == KIND_SKIP) continue;
            const int64_t lo = (int64_t)d.out_off - base + (int64_t)d.pre_end * d.out_nch;
            const int64_t hi = (int64_t)d.out_off - base + (int64_t)d.nframes * d.out_nch;
            if (lo < 0 || hi > ext) (*bad_reserved)++;
            if (lo < 0 || hi > vals) (*bad_values)++;
        }
        base += ext;
    }
}

// Returns frames (or -2 open error, -3 exception); fills out (cap ints).
// seek_to >= 0: as a caller that calls SetSample(seek_to) first (*seek_rc: its result).
int64_t emu_decode_from(const uint8_t *file, size_t len, int64_t seek_to, int chunk, int32_t *out, int64_t cap,
                        int64_t *crc_errors, int *nch, uint32_t *status_or, int *seek_rc) {
    FramingOutput fo;
    FileInfo info;
    fo.defer_values = true;  // as the product path: the metadata values come from meta_apply
    frame_file(file, len, 0, 0, 0, chunk, fo, info, seek_to);
    apply_meta_jobs(fo, file);
    *seek_rc = info.seek_result;
    *crc_errors = 0;
    *status_or = 0;
    *nch = info.out_nch;
    if (!info.open_ok) return -2;
    int64_t total = info.out_frames * info.out_nch;
    if (total > cap) return -4;
    memset(out, 0, sizeof(int32_t) * (size_t)total);
    std::vector<int32_t> ptable(256);
    bool exception = info.exception != 0;
    std::vector<std::pair<int64_t, int64_t>> fills;
    PcmState chain;  // the state a chain carries from block to block (wv_decode_chain)
    DsdState dchain;  // ... and a DSD chain (decode_dsd_chain)
    for (auto &d : fo.descs) {
        uint32_t st = d.fstatus;
        HostStore hs{out, d.out_off, (uint64_t)d.pre_end * d.out_nch};
        if (d.kind == KIND_PCM && (d.chain_len || (d.inherit & INH_MEMBER))) {
            st |= pcm_state_load(chain, d, file);
            st |= decode_pcm_run<HostStore, true>(chain, d, hs, nullptr);
        } else if (d.kind == KIND_PCM) {
            st |= decode_pcm_block(d, file, hs);
        } else if (d.kind != KIND_SKIP) {
            DsdResult r = (d.chain_len || (d.inherit & INH_MEMBER))
                              ? decode_dsd_chained(dchain, d, d.chain_len != 0, file, fo.tables.data(), ptable.data(), hs)
                              : decode_dsd_block(d, file, fo.tables.data(), ptable.data(), hs);
            st |= r.status;
            if (r.status & ST_DSD_MUTE) {
                // chunks from mute_chunk on: fill n*call_nch from the call start (a false-stereo
                // block's final call that failed its CRC first goes back to one value per
                // frame: wv_dsd_fill / dsd_fs_unexpand)
                const bool fs = (d.flags & wvf::FALSE_STEREO) && !(d.flags & wvf::MONO_FLAG) &&
                                d.nframes == d.block_samples;
                uint32_t f = 0, cl = d.first_chunk;
                for (uint32_t ci = 0; f < d.nframes; ci++) {
                    uint32_t n = cl < d.nframes - f ? cl : d.nframes - f;
                    if (ci >= r.mute_chunk && f >= d.pre_end) {
                        if (fs && ci == r.mute_chunk && f + n == d.nframes) {
                            const int64_t p = (int64_t)d.out_off + (int64_t)f * d.out_nch;
                            for (int64_t k = 0; k < (int64_t)n; k++) out[p + k] = out[p + 2 * k];
                            if (f == 0 && d.first_bsp > 0) st |= ST_NONDET;
                        }
                        int64_t start = (int64_t)d.out_off + (int64_t)f * d.out_nch - (ci == 0 ? d.first_bsp : 0);
                        fills.push_back({start, (int64_t)n * d.call_nch});
                    }
                    f += n;
                    cl = next_call_len(d, f);
                }
            }
        }
        // a block decoded from state the device cannot see (malformed files only):
        // the reference decodes garbage and its CRC check fails (as wv_api.cpp)
        if ((st & ST_UNSUPPORTED) && d.nframes == d.block_samples) st |= ST_CRC_CHECKED | ST_CRC_ERROR;
        *status_or |= st;
        if (st & ST_CRC_ERROR) (*crc_errors)++;
        if (st & ST_EXCEPTION) {
            exception = true;
            break;
        }
    }
    for (auto &fl : fills)
        for (int64_t i = 0; i < fl.second; i++) out[fl.first + i] = 0x55;
    if (exception) return -3;
    return info.out_frames;
}

// A hybrid file with its .wvc correction file (wvc_len 0: none), opened with
// open_flags, decoded by the device core on the host (blocks in order, no
// chains): frames or -2/-3, as emu_decode.
int64_t emu_decode_wvc(const uint8_t *file, size_t len, const uint8_t *wvc, size_t wvc_len, int chunk,
                       uint32_t open_flags, int32_t *out, int64_t cap, int64_t *crc_errors, int *nch,
                       uint32_t *status_or) {
    std::vector<uint8_t> blob(len + wvc_len + 64, 0xFF);
    memcpy(blob.data(), file, len);
    if (wvc_len) memcpy(blob.data() + len, wvc, wvc_len);
    FramingOutput fo;
    FileInfo info;
    fo.defer_values = true;
    frame_file(blob.data(), len, 0, 0, open_flags, chunk, fo, info, -1, wvc_len ? blob.data() + len : nullptr,
               wvc_len, len);
    apply_meta_jobs(fo, blob.data());
    *crc_errors = 0;
    *status_or = 0;
    *nch = info.out_nch;
    if (!info.open_ok) return -2;
    const int64_t total = info.out_frames * info.out_nch;
    if (total > cap) return -4;
    memset(out, 0, sizeof(int32_t) * (size_t)total);
    for (auto &d : fo.descs) {
        if (d.kind != KIND_PCM || d.chain_len || (d.inherit & INH_MEMBER)) return -5;
        HostStore hs{out, d.out_off, (uint64_t)d.pre_end * d.out_nch};
        uint32_t st = d.fstatus | decode_pcm_block(d, blob.data(), hs);
        // bit 16: a block read its correction stream; bit 17: an exact-float block read a wvx stream
        *status_or |= st | (d.wvc_len ? 0x10000u : 0u) | ((d.xfloat && (d.wvx_state & 1)) ? 0x20000u : 0u);
        if (st & ST_CRC_ERROR) (*crc_errors)++;
        if (st & ST_EXCEPTION) return -3;
    }
    return info.out_frames;
}

int64_t emu_decode(const uint8_t *file, size_t len, int chunk, int32_t *out, int64_t cap, int64_t *crc_errors,
                   int *nch, uint32_t *status_or) {
    int seek_rc = 0;
    return emu_decode_from(file, len, -1, chunk, out, cap, crc_errors, nch, status_or, &seek_rc);
}

// Descriptors of one file (bytes, BlockDesc after BlockDesc), framed with the
// metadata values on the host (defer = 0) or deferred and applied by meta_apply
// (defer = 1); returns the descriptor count (or -4: cap too small).
int64_t emu_frame_descs(const uint8_t *file, size_t len, int64_t seek_to, int chunk, int defer, void *out,
                        int64_t cap_bytes, int64_t *njobs) {
    FramingOutput fo;
    FileInfo info;
    fo.defer_values = defer != 0;
    frame_file(file, len, 0, 0, 0, chunk, fo, info, seek_to);
    *njobs = (int64_t)fo.jobs.size();
    if (defer) apply_meta_jobs(fo, file);
    int64_t nb = (int64_t)(fo.descs.size() * sizeof(BlockDesc));
    if (nb > cap_bytes) return -4;
    if (nb) memcpy(out, fo.descs.data(), (size_t)nb);
    return (int64_t)fo.descs.size();
}

static int info_vals(const FileInfo &info, int64_t ndesc, int64_t *vals, int nvals) {
    int64_t v[] = {info.open_ok, info.total_samples, info.sample_rate, info.num_channels, info.bits_per_sample,
                   info.bytes_per_sample, info.reduced_channels, info.mode, info.version, info.is_float,
                   info.out_frames, info.out_nch, ndesc, (int64_t)info.dsd_multiplier,
                   info.lossy_blocks, info.is_five, info.file_format, info.header_off, info.header_len,
                   info.trailer_off, info.trailer_len, info.first_call_frames, info.config_flags,
                   info.sample_index0, info.exception, info.nondet};
    int n = (int)(sizeof(v) / sizeof(v[0]));
    for (int i = 0; i < n && i < nvals; i++) vals[i] = v[i];
    return n;
}

// FileInfo fields of the host framing, for the WavpackGet* getters' tests.
int emu_file_info_chunk(const uint8_t *file, size_t len, int chunk, int64_t *vals, int nvals) {
    FramingOutput fo;
    FileInfo info;
    frame_file(file, len, 0, 0, 0, chunk, fo, info);
    return info_vals(info, (int64_t)fo.descs.size(), vals, nvals);
}
int emu_file_info(const uint8_t *file, size_t len, int64_t *vals, int nvals) {
    return emu_file_info_chunk(file, len, 4096, vals, nvals);
}

// The device framing (wv_dframe.h) run on the host, one file: the walk, every
// block's descriptor, the host-side FileInfo reduction.  Returns the block
// count, or -(1 + why) when the file is left to the host framing (*why: the
// DF_* reason, 9 = the blocks' records disagree).
int64_t emu_dframe(const uint8_t *file, size_t len, int chunk, void *descs, int64_t cap_bytes, int64_t *vals,
                   int nvals) {
    DFile df;
    memset(&df, 0, sizeof(df));
    df.base = 0;
    df.len = len;
    df.slot = 0;
    df.chunk = (uint32_t)chunk;
    std::vector<uint64_t> slots(len / 32 + 1);
    dframe_walk(df, file, slots.data());
    if (!df.regular) return -1 - (int64_t)df.why;
    std::vector<BlockDesc> d(df.nblocks);
    std::vector<DBlock> r(df.nblocks);
    df.out_base = 0;
    df.first_desc = 0;
    for (uint32_t k = 0; k < df.nblocks; k++) dframe_block(df, k, file, slots.data(), d[k], r[k]);
    FileInfo fi;
    if (!dframe_file_info(df, r.data(), fi)) {
        for (uint32_t k = 0; k < df.nblocks; k++)
            if (!r[k].regular) return -1 - (int64_t)r[k].why;
        return -1 - (int64_t)DF_UNIFORM;
    }
    const int64_t nb = (int64_t)(d.size() * sizeof(BlockDesc));
    if (nb > cap_bytes) return -100;
    memcpy(descs, d.data(), (size_t)nb);
    info_vals(fi, (int64_t)df.nblocks, vals, nvals);
    return (int64_t)df.nblocks;
}
}
