// wv_api.cpp -- the C-ABI (include/wvgpu.h) over the framing and the HIP kernels.
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/wvgpu.h"
#include "wv_desc.h"
#include "wv_format.h"
#include "wv_framing.h"

namespace wvg {
hipError_t launch_decode(const BlockDesc *descs, const uint32_t *pcm_list, uint32_t n_pcm, const uint32_t *dsd_list,
                         uint32_t n_dsd, const uint8_t *blob, const uint8_t *tables, int32_t *ptables, int32_t *out,
                         uint32_t *status, uint32_t *mute_chunk, hipStream_t s);
int term_set_of(const BlockDesc &d);
hipError_t launch_2wave(int ts, const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                        int32_t *out, uint32_t *status, hipStream_t s);
constexpr int kMaxTermSets = 8;
}

using namespace wvg;

struct wvg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
};

struct wvg_batch {
    wvg_ctx *ctx = nullptr;
    int chunk = 4096;
    std::vector<uint8_t> blob;
    FramingOutput fo;
    std::vector<FileInfo> finfo;
    std::vector<wvg_file_info> infos;
    int64_t out_ints = 0;
    std::vector<uint32_t> pcm_list, dsd_list;           // lane kernels (generic PCM, DSD)
    std::vector<uint32_t> ts_list[kMaxTermSets];        // two-wave kernels per term set
    uint32_t *d_ts[kMaxTermSets] = {nullptr};
    int force_lane = 0;                                 // WVG_FORCE_LANE=1: everything on the lane kernel
    std::vector<uint32_t> h_status;
    int64_t bytes_in = 0, frames = 0;
    // device
    uint8_t *d_blob = nullptr, *d_tables = nullptr;
    BlockDesc *d_descs = nullptr;
    int32_t *d_out = nullptr, *d_ptables = nullptr;
    uint32_t *d_status = nullptr, *d_mute = nullptr, *d_pcm = nullptr, *d_dsd = nullptr;
    bool uploaded = false, downloaded = false;
};

static int hip_fail(wvg_ctx *c, hipError_t e, const char *what) {
    if (c) c->err = std::string(what) + ": " + hipGetErrorString(e);
    return WVG_ERR_HIP;
}
#define HIPCHK(c, x)                                          \
    do {                                                      \
        hipError_t _e = (x);                                  \
        if (_e != hipSuccess) return hip_fail((c), _e, #x); \
    } while (0)

extern "C" {

wvg_ctx *wvg_open(int device) {
    wvg_ctx *c = new wvg_ctx();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        delete c;
        return nullptr;
    }
    if (device < 0) hipGetDevice(&device);
    if (hipSetDevice(device) != hipSuccess) {
        delete c;
        return nullptr;
    }
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return nullptr;
    }
    return c;
}

void wvg_close(wvg_ctx *c) {
    if (!c) return;
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

const char *wvg_last_error(wvg_ctx *c) { return c ? c->err.c_str() : "no context"; }

wvg_batch *wvg_batch_new(wvg_ctx *c, int chunk_frames) {
    if (!c || chunk_frames <= 0) return nullptr;
    wvg_batch *b = new wvg_batch();
    b->ctx = c;
    b->chunk = chunk_frames;
    const char *fl = getenv("WVG_FORCE_LANE");
    b->force_lane = fl && fl[0] == '1';
    return b;
}

static void free_dev(wvg_batch *b) {
    hipFree(b->d_blob);
    hipFree(b->d_tables);
    hipFree(b->d_descs);
    hipFree(b->d_out);
    hipFree(b->d_ptables);
    hipFree(b->d_status);
    hipFree(b->d_mute);
    hipFree(b->d_pcm);
    hipFree(b->d_dsd);
    for (int t = 0; t < kMaxTermSets; t++) {
        hipFree(b->d_ts[t]);
        b->d_ts[t] = nullptr;
    }
    b->d_blob = b->d_tables = nullptr;
    b->d_descs = nullptr;
    b->d_out = b->d_ptables = nullptr;
    b->d_status = b->d_mute = b->d_pcm = b->d_dsd = nullptr;
    b->uploaded = false;
}

void wvg_batch_free(wvg_batch *b) {
    if (!b) return;
    hipSetDevice(b->ctx->device);
    free_dev(b);
    delete b;
}

// FileInfo -> the getters' view (WavPackUtils.cs:346-499 applied here, once)
static void fill_info(const FileInfo &fi, wvg_file_info &wi) {
    memset(&wi, 0, sizeof(wi));
    wi.open_ok = fi.open_ok;
    strncpy(wi.error, fi.error.c_str(), sizeof(wi.error) - 1);
    wi.num_channels = fi.num_channels != 0 ? fi.num_channels : 2;
    wi.reduced_channels = fi.out_nch;
    wi.bits_per_sample = fi.bits_per_sample ? (fi.dsd_multiplier > 0 ? fi.bits_per_sample / 8 : fi.bits_per_sample) : 16;
    wi.bytes_per_sample = fi.bytes_per_sample ? fi.bytes_per_sample : 2;
    wi.version = fi.version;
    wi.mode = fi.mode;
    wi.is_float = fi.is_float;
    wi.is_five = fi.is_five;
    wi.file_format = fi.file_format;
    wi.lossy = ((fi.config_flags & 8) != 0) || (fi.mode & 0x4) != 0 || (fi.open_ok && !(fi.mode & 0x2) && !(fi.mode & 0x4) && fi.lossy_blocks);
    wi.dsd_multiplier = fi.dsd_multiplier;
    wi.sample_rate = fi.sample_rate ? (fi.dsd_multiplier > 0 ? (int64_t)fi.dsd_multiplier * fi.sample_rate * 8 : fi.sample_rate) : 44100;
    wi.total_samples = fi.total_samples;
    wi.out_frames = fi.out_frames;
    wi.out_offset = 0;
}

int wvg_probe_file(const uint8_t *file, size_t len, uint32_t open_flags, int chunk_frames, wvg_file_info *info) {
    if ((!file && len) || !info) return WVG_ERR_ARG;
    FramingOutput fo;
    FileInfo fi;
    frame_file(file, len, 0, 0, open_flags, chunk_frames > 0 ? chunk_frames : 4096, fo, fi);
    fill_info(fi, *info);
    return fi.open_ok ? WVG_OK : WVG_ERR_OPEN;
}

int wvg_batch_add_file(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, wvg_file_info *info) {
    if (!b || (!file && len)) return WVG_ERR_ARG;
    if (b->uploaded) free_dev(b);
    size_t base = (b->blob.size() + 15) & ~(size_t)15;
    b->blob.resize(base + len);
    if (len) memcpy(b->blob.data() + base, file, len);
    FileInfo fi;
    frame_file(b->blob.data() + base, len, base, (uint64_t)b->out_ints, open_flags, b->chunk, b->fo, fi);
    wvg_file_info wi;
    fill_info(fi, wi);
    wi.out_offset = b->out_ints;
    wi.header_off = fi.header_off;
    wi.header_len = fi.header_len;
    wi.trailer_off = fi.trailer_off;
    wi.trailer_len = fi.trailer_len;
    b->finfo.push_back(fi);
    b->infos.push_back(wi);
    if (info) *info = wi;
    if (!fi.open_ok) return WVG_ERR_OPEN;
    b->out_ints += fi.out_frames * fi.out_nch;
    for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++) {
        const BlockDesc &d = b->fo.descs[(size_t)k];
        int ts = (d.kind == KIND_PCM && !b->force_lane) ? term_set_of(d) : -1;
        if (ts >= 0) b->ts_list[ts].push_back((uint32_t)k);
        else if (d.kind == KIND_PCM) b->pcm_list.push_back((uint32_t)k);
        else if (d.kind != KIND_SKIP) b->dsd_list.push_back((uint32_t)k);
        b->frames += d.nframes;
    }
    // compressed bytes of the file's decoded blocks (whole file is a fine proxy)
    b->bytes_in += (int64_t)len;
    return (int)b->infos.size() - 1;
}

int wvg_batch_upload(wvg_batch *b) {
    if (!b) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    free_dev(b);
    size_t blob_n = b->blob.size() + 64;
    HIPCHK(c, hipMalloc(&b->d_blob, blob_n));
    HIPCHK(c, hipMemsetAsync(b->d_blob, 0xFF, blob_n, c->stream));
    if (!b->blob.empty()) HIPCHK(c, hipMemcpyAsync(b->d_blob, b->blob.data(), b->blob.size(), hipMemcpyHostToDevice, c->stream));
    size_t nd = b->fo.descs.size();
    HIPCHK(c, hipMalloc(&b->d_descs, sizeof(BlockDesc) * (nd ? nd : 1)));
    if (nd) HIPCHK(c, hipMemcpyAsync(b->d_descs, b->fo.descs.data(), sizeof(BlockDesc) * nd, hipMemcpyHostToDevice, c->stream));
    size_t nt = b->fo.tables.size() + 16;
    HIPCHK(c, hipMalloc(&b->d_tables, nt));
    if (!b->fo.tables.empty())
        HIPCHK(c, hipMemcpyAsync(b->d_tables, b->fo.tables.data(), b->fo.tables.size(), hipMemcpyHostToDevice, c->stream));
    size_t no = (size_t)(b->out_ints ? b->out_ints : 1);
    HIPCHK(c, hipMalloc(&b->d_out, sizeof(int32_t) * no));
    HIPCHK(c, hipMemsetAsync(b->d_out, 0, sizeof(int32_t) * no, c->stream));
    HIPCHK(c, hipMalloc(&b->d_status, sizeof(uint32_t) * (nd ? nd : 1)));
    HIPCHK(c, hipMalloc(&b->d_mute, sizeof(uint32_t) * (nd ? nd : 1)));
    std::vector<uint32_t> st(nd ? nd : 1);
    for (size_t k = 0; k < nd; k++) st[k] = b->fo.descs[k].fstatus;
    HIPCHK(c, hipMemcpyAsync(b->d_status, st.data(), sizeof(uint32_t) * st.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(b->d_mute, 0, sizeof(uint32_t) * (nd ? nd : 1), c->stream));
    size_t np = b->pcm_list.size(), ns = b->dsd_list.size();
    HIPCHK(c, hipMalloc(&b->d_pcm, sizeof(uint32_t) * (np ? np : 1)));
    HIPCHK(c, hipMalloc(&b->d_dsd, sizeof(uint32_t) * (ns ? ns : 1)));
    if (np) HIPCHK(c, hipMemcpyAsync(b->d_pcm, b->pcm_list.data(), sizeof(uint32_t) * np, hipMemcpyHostToDevice, c->stream));
    if (ns) HIPCHK(c, hipMemcpyAsync(b->d_dsd, b->dsd_list.data(), sizeof(uint32_t) * ns, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMalloc(&b->d_ptables, sizeof(int32_t) * 256 * (ns ? ns : 1)));
    for (int t = 0; t < kMaxTermSets; t++) {
        size_t nl = b->ts_list[t].size();
        if (!nl) continue;
        HIPCHK(c, hipMalloc(&b->d_ts[t], sizeof(uint32_t) * nl));
        HIPCHK(c, hipMemcpyAsync(b->d_ts[t], b->ts_list[t].data(), sizeof(uint32_t) * nl, hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    b->uploaded = true;
    b->downloaded = false;
    return WVG_OK;
}

int wvg_batch_decode(wvg_batch *b, void *stream) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    for (int t = 0; t < kMaxTermSets; t++)
        if (!b->ts_list[t].empty())
            HIPCHK(c, launch_2wave(t, b->d_descs, b->d_ts[t], (uint32_t)b->ts_list[t].size(), b->d_blob, b->d_out,
                                   b->d_status, s));
    HIPCHK(c, launch_decode(b->d_descs, b->d_pcm, (uint32_t)b->pcm_list.size(), b->d_dsd, (uint32_t)b->dsd_list.size(),
                            b->d_blob, b->d_tables, b->d_ptables, b->d_out, b->d_status, b->d_mute, s));
    b->downloaded = false;
    return WVG_OK;
}

int wvg_batch_sync(wvg_batch *b) {
    if (!b) return WVG_ERR_ARG;
    HIPCHK(b->ctx, hipStreamSynchronize(b->ctx->stream));
    HIPCHK(b->ctx, hipDeviceSynchronize());
    return WVG_OK;
}

int64_t wvg_batch_out_ints(const wvg_batch *b) { return b ? b->out_ints : 0; }
int32_t *wvg_batch_device_out(wvg_batch *b) { return b ? b->d_out : nullptr; }
int64_t wvg_batch_num_blocks(const wvg_batch *b) { return b ? (int64_t)b->fo.descs.size() : 0; }
int64_t wvg_batch_bytes_in(const wvg_batch *b) { return b ? b->bytes_in : 0; }
int64_t wvg_batch_frames(const wvg_batch *b) { return b ? b->frames : 0; }

int wvg_batch_download(wvg_batch *b, int32_t *host_out, int64_t cap_ints) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipDeviceSynchronize());
    if (host_out) {
        if (cap_ints < b->out_ints) return WVG_ERR_SPACE;
        if (b->out_ints)
            HIPCHK(c, hipMemcpy(host_out, b->d_out, sizeof(int32_t) * (size_t)b->out_ints, hipMemcpyDeviceToHost));
    }
    size_t nd = b->fo.descs.size();
    b->h_status.assign(nd, 0);
    if (nd) HIPCHK(c, hipMemcpy(b->h_status.data(), b->d_status, sizeof(uint32_t) * nd, hipMemcpyDeviceToHost));
    b->downloaded = true;
    return WVG_OK;
}

int wvg_batch_block_status(wvg_batch *b, uint32_t *out, int64_t cap) {
    if (!b || !b->downloaded) return WVG_ERR_ARG;
    int64_t n = (int64_t)b->h_status.size();
    if (cap < n) return WVG_ERR_SPACE;
    if (n) memcpy(out, b->h_status.data(), sizeof(uint32_t) * (size_t)n);
    return (int)n;
}

int wvg_batch_file_result(wvg_batch *b, int file, wvg_file_result *res) {
    if (!b || !b->downloaded || file < 0 || file >= (int)b->finfo.size() || !res) return WVG_ERR_ARG;
    const FileInfo &fi = b->finfo[(size_t)file];
    memset(res, 0, sizeof(*res));
    res->frames = fi.out_frames;
    res->exception = fi.exception;
    res->num_blocks = (int32_t)fi.num_desc;
    res->lossy = fi.lossy_blocks || (fi.config_flags & 8) != 0;
    for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++) {
        const BlockDesc &d = b->fo.descs[(size_t)k];
        uint32_t st = b->h_status[(size_t)k];
        // a block decoded from state the device cannot see (only in malformed
        // files): the reference decodes garbage and its CRC check fails
        if ((st & ST_UNSUPPORTED) && d.nframes == d.block_samples) st |= ST_CRC_CHECKED | ST_CRC_ERROR;
        res->status_or |= st;
        if (st & ST_CRC_ERROR) res->crc_errors++;
        if (st & ST_EXCEPTION) {
            res->exception = 1;
            break;
        }
    }
    if (res->exception) res->frames = -1;
    return WVG_OK;
}

int wvg_batch_time(wvg_batch *b, int iters, float *ms) {
    // mean device time of one decode launch: an event pair around each launch on
    // the decode stream, so launch gaps between iterations are not counted
    if (!b || !b->uploaded || iters <= 0) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    std::vector<hipEvent_t> ev((size_t)iters * 2);
    for (auto &e : ev) HIPCHK(c, hipEventCreate(&e));
    for (int i = 0; i < iters; i++) {
        HIPCHK(c, hipEventRecord(ev[2 * i], c->stream));
        int rc = wvg_batch_decode(b, nullptr);
        if (rc) return rc;
        HIPCHK(c, hipEventRecord(ev[2 * i + 1], c->stream));
    }
    HIPCHK(c, hipEventSynchronize(ev.back()));
    double tot = 0;
    for (int i = 0; i < iters; i++) {
        float t = 0;
        HIPCHK(c, hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
        tot += t;
    }
    for (auto &e : ev) hipEventDestroy(e);
    *ms = (float)(tot / iters);
    return WVG_OK;
}

int wvg_decode_file(wvg_ctx *ctx, const uint8_t *file, size_t len, int chunk_frames, int32_t *out, int64_t cap_ints,
                    wvg_file_info *info, wvg_file_result *res) {
    wvg_batch *b = wvg_batch_new(ctx, chunk_frames);
    if (!b) return WVG_ERR_ARG;
    int fi = wvg_batch_add_file(b, file, len, 0, info);
    if (fi < 0) {
        wvg_batch_free(b);
        return fi;
    }
    int rc = wvg_batch_upload(b);
    if (!rc) rc = wvg_batch_decode(b, nullptr);
    if (!rc) rc = wvg_batch_download(b, out, cap_ints);
    if (!rc) rc = wvg_batch_file_result(b, fi, res);
    wvg_batch_free(b);
    return rc;
}

int wvg_format_samples(const int32_t *src, int64_t samcnt, int bps, uint8_t *pcm, int64_t pcm_len, int offset, int dsd) {
    // WavPackUtils.cs:288-341
    int64_t len = samcnt * bps, counter = offset, c2 = 0;
    if (!pcm || pcm_len < len + offset) return 0;
    switch (bps) {
    case 1:
        if (dsd)
            while (samcnt-- > 0) pcm[counter++] = (uint8_t)src[c2++];
        else
            while (samcnt-- > 0) pcm[counter++] = (uint8_t)(0xFF & (src[c2++] + 128));
        break;
    case 2:
        while (samcnt-- > 0) {
            int32_t t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
        }
        break;
    case 3:
        while (samcnt-- > 0) {
            int32_t t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
            pcm[counter++] = (uint8_t)(t >> 16);
        }
        break;
    case 4:
        while (samcnt-- > 0) {
            int32_t t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
            pcm[counter++] = (uint8_t)(t >> 16);
            pcm[counter++] = (uint8_t)((uint32_t)t >> 24);
        }
        break;
    }
    return 1;
}

}  // extern "C"
