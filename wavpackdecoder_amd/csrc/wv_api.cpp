// wv_api.cpp -- the C-ABI (include/wvgpu.h) over the framing and the HIP kernels.
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstddef>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wvgpu.h"
#include "wv_desc.h"
#include "wv_format.h"
#include "wv_framing.h"

namespace wvg {
hipError_t launch_decode(const BlockDesc *descs, const uint32_t *pcm_list, uint32_t n_pcm, const uint32_t *dsd_list,
                         uint32_t n_dsd, uint32_t fast_lo, uint32_t n_fast, const uint8_t *blob, const uint8_t *tables,
                         int32_t *out, uint32_t *status, uint32_t *aux, hipStream_t s_pcm, hipStream_t s_dsd,
                         hipStream_t s_fast, int lane_mode, uint32_t high_lo, uint32_t n_high_mono,
                         int lane_mode_fast, uint32_t n_fast_mono, int lane_mode_wvc, uint32_t n_pcm_wvc);
bool wvc_lane_candidate(const BlockDesc &d);
int term_set_of(const BlockDesc &d, int prefer_pipe);
bool lane_rt_group(int ts);  // the launch groups of the run-time list lane kernel (wv_pcm_lane_rt)
hipError_t launch_2wave(int ts, const BlockDesc *descs, const uint32_t *list, uint32_t n, const uint8_t *blob,
                        int32_t *out, uint32_t *status, uint32_t *aux, hipStream_t s, int lane_mode,
                        const uint32_t *lane_list, uint32_t lane_n, uint32_t *lane_dbg);
hipError_t launch_format(const FormatSeg *segs, uint32_t nseg, const int32_t *in, uint8_t *out, int dsd, hipStream_t s);
hipError_t launch_copy_to_host(const uint8_t *src, uint8_t *dst, size_t n, hipStream_t s);
hipError_t launch_zero_fill(const ZeroSeg *segs, uint32_t nseg, int32_t *out, hipStream_t s);
hipError_t upload_dsd_ptables();
hipError_t launch_dsd_fill(const BlockDesc *descs, const uint32_t *dsd_list, uint32_t n_dsd, uint32_t *status,
                           const uint32_t *aux, int32_t *out, hipStream_t s);
hipError_t launch_dframe_rank(DFile *files, const uint32_t *tile_file, uint32_t ntiles, const uint32_t *rank_files,
                              uint32_t nrank, const uint8_t *blob, uint32_t *cand, uint32_t cand_cap, uint32_t *cnt,
                              uint64_t *slots, hipStream_t s);
size_t dframe_tile_cap();
size_t dframe_tile_bytes();
hipError_t launch_dframe_walk(DFile *files, uint32_t n, const uint8_t *blob, uint64_t *slots, hipStream_t s);
hipError_t launch_dframe_block(const DFile *files, const uint32_t *blk_file, const uint32_t *blk_k, uint32_t n,
                               const uint8_t *blob, const uint64_t *slots, BlockDesc *descs, DBlock *recs,
                               hipStream_t s);
hipError_t launch_meta(BlockDesc *descs, const MetaJob *jobs, uint32_t njobs, const MetaItem *items, const uint8_t *blob,
                       hipStream_t s);
constexpr int kMaxTermSets = 8;
constexpr size_t kLaneDbgWaves = 4096;  // lane-kernel counters (WVG_LANE_COUNTERS): parser waves per term set
constexpr uint32_t kFormatSeg = 65536;  // values per format work item
}

using namespace wvg;

// The kernels of one decode (a two-wave launch per term set, the generic PCM
// kernel, the DSD kernels) are independent: they fork from the batch's stream
// onto the batch's side streams and join back, so small groups run concurrently.
// Every batch owns its streams, so batches of one context (or of several host
// threads) run concurrently on the device; nothing synchronises the whole device.
constexpr int kSide = kMaxTermSets + 3;  // term sets, generic PCM, DSD, DSD mode 1
// streams one decode launches on, at most (WVG_LANES: fewer): its batch's stream and the
// context's side streams.  Every stream takes one of the process's few hardware queues
// (GPU_MAX_HW_QUEUES), and two busy streams on one queue run one after another, so the
// side streams are few and shared by the context's batches (a decode uses them only
// when no other batch of the context is running): with N batches in flight the process
// holds N + 2 streams.  Three lanes give a mixed batch its latency (C5: DSD mode 3,
// DSD mode 1 and the PCM groups side by side, 54.6 ms, as with a lane per group).
constexpr int kLanes = 3;
constexpr size_t kAutoLaneMin = 2048;  // WVG_KERNEL_AUTO: larger groups decode on lanes even alone
// how long a context keeps the lane kernels after batches last overlapped (a caller that
// keeps several batches in flight issues its next decode well within it; one that went
// back to a batch at a time gets the latency kernels again after it)
constexpr double kConcurrentHoldMs = 1000.0;
// The part of a device-framed descriptor the host reads (kind, flags, frames, the
// call schedule, status, terms): everything up to and including term[].  The rest
// (weights, histories, DSD, seek, sticky, .wvc, exact float) is zero or unused on
// the host for the files the device framer accepts.
constexpr size_t kDescHead = offsetof(BlockDesc, term) + sizeof(((BlockDesc *)nullptr)->term);
constexpr int SAMPLE_BUFFER_SIZE = 4096;  // Defines.cs:18, the request size WvDemo uses
constexpr size_t kTimingPending = 64;  // timing pairs left pending before the oldest is folded

struct wvg_batch;
struct wvg_ctx {
    int device = 0;
    std::string err;
    std::mutex mu;                   // guards `batches` and `side`
    std::vector<wvg_batch *> batches;  // live batches (a decode counts those still running)
    hipStream_t side[kLanes - 1] = {nullptr};  // side streams: lanes 1 .. kLanes - 1 of a decode
    // when a decode last found another batch of this context running (now_ms; WVG_KERNEL_AUTO
    // keeps the lane kernels for kConcurrentHoldMs after it)
    std::atomic<double> concurrent_ms{-1e30};
    // the process's hardware queues (GPU_MAX_HW_QUEUES as the process started; HIP's default
    // 4): the stream budget the batches in flight share (wvg_batch_decode's own-stream policy)
    int hw_queues = 4;
    // WVG_DSD_STREAM: 0 never give a batch streams of its own while others run, 1 always
    // (two), unset: as many as the queue budget leaves each batch in flight (up to kLanes)
    int own_streams = -1;
};

// Page-locked, grow-only host buffer: the batch's file bytes live here from
// add_file on, so the upload is one DMA at PCIe rate (no pageable staging), and
// the decoded output can be downloaded into one (wvg_batch_host_out).
struct PinnedBuf {
    uint8_t *p = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf &) = delete;
    PinnedBuf &operator=(const PinnedBuf &) = delete;
    ~PinnedBuf() { release(); }
    void release() {
        if (p) {
            if (pinned) hipHostFree(p);
            else free(p);
        }
        p = nullptr;
        n = cap = 0;
    }
    bool reserve(size_t m) {
        if (m <= cap) return true;
        size_t nc = cap ? cap : (size_t)1 << 20;
        while (nc < m) nc *= 2;
        uint8_t *q = nullptr;
        bool pin = hipHostMalloc((void **)&q, nc, hipHostMallocDefault) == hipSuccess;
        if (!pin) q = (uint8_t *)malloc(nc);  // no device memory for page-locking: plain pages
        if (!q) return false;
        if (n) memcpy(q, p, n);
        const size_t keep = n;
        release();
        p = q;
        cap = nc;
        n = keep;
        pinned = pin;
        return true;
    }
    bool resize(size_t m) {
        if (!reserve(m)) return false;
        n = m;
        return true;
    }
    uint8_t *data() { return p; }
    const uint8_t *data() const { return p; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
};

struct wvg_batch {
    wvg_ctx *ctx = nullptr;
    int chunk = 4096;
    hipStream_t stream = nullptr;          // the batch's own stream (default for decode/format/download)
    hipEvent_t fork = nullptr, join[kLanes - 1] = {nullptr};  // lanes 1 .. (the context's side streams)
    hipStream_t dstream[2] = {nullptr, nullptr};  // the batch's own side streams while others run (own_side)
    hipEvent_t done = nullptr;             // end of the last decode/format, on whatever stream it ran
    hipEvent_t up = nullptr;               // end of the last upload's copies (on the batch stream)
    bool timing = false;                   // wvg_batch_set_timing: an event pair around every decode
    std::vector<hipEvent_t> tev;           // pending (start, end) pairs, folded into t_sum/t_cnt
    std::vector<hipEvent_t> tfree;         // event objects of folded pairs, reused
    // timing on: the end of each launch group of the last decode, on its own
    // stream (wvg_batch_group_times), against that decode's start event
    hipEvent_t gev[kSide] = {nullptr};
    hipEvent_t gstart = nullptr;
    uint32_t gmask = 0;                    // groups the last timed decode launched
    double t_sum = 0;
    int t_cnt = 0;
    // device buffers are kept across uploads and only grown (capacities in bytes)
    size_t cap_blob = 0, cap_descs = 0, cap_items = 0, cap_jobs = 0, cap_tables = 0, cap_out = 0, cap_st = 0,
           cap_pcml = 0, cap_dsd = 0, cap_pcm = 0, cap_segs = 0, cap_ts[kMaxTermSets] = {0};
    bool segs_uploaded = false;
    PinnedBuf blob;                                     // every file's bytes, 16-B aligned
    // the blob goes to the device as it is filled (blob_push): bytes [0, blob_dev)
    // are in d_blob already, and a DMA from the page-locked blob may be running
    size_t blob_dev = 0;
    bool blob_dma = false;
    PinnedBuf hout;                                     // wvg_batch_host_out: the output, downloaded
    PinnedBuf stage;                                    // page-locked copies of an upload's small host arrays
    PinnedBuf hst;                                      // page-locked landing area of the status download
    PinnedBuf hpcm;                                     // wvg_batch_host_pcm: the formatted PCM, downloaded
    FramingOutput fo;
    std::vector<FileInfo> finfo;
    std::vector<wvg_file_info> infos;
    int64_t out_ints = 0;
    std::vector<uint32_t> pcm_list, dsd_list;           // wave-per-block kernels (generic PCM, DSD)
    uint32_t dsd_fast_lo = 0, dsd_fast_n = 0;          // the mode-1 range of dsd_list (sorted by kind)
    uint32_t dsd_fast_mono = 0;                        // ... its mono blocks (after the stereo ones)
    uint32_t pcm_wvc_n = 0;                            // pcm_list's tail: .wvc lane candidates
    uint32_t dsd_high_lo = 0, dsd_high_mono = 0;       // the mode-3 range [high_lo, end): stereo, then mono blocks
    std::vector<uint32_t> ts_list[kMaxTermSets];        // two-wave kernels per term set
    int64_t gframes[kSide] = {0};                       // frames per launch group (the lane assignment's load)
    uint32_t *d_ts[kMaxTermSets] = {nullptr};      // per term set: the list, then the lane kernels' order of it
    std::vector<uint32_t> ts_lane[kMaxTermSets];  // the lane order (kLaneGap entries included)
    uint32_t *d_lane_dbg = nullptr;               // WVG_LANE_COUNTERS=1: per parser wave cycles + groups by path
    int force_lane = 0;                                 // WVG_FORCE_LANE=1: every PCM block on the generic kernel
    int prefer_pipe = 0;                                // WVG_PIPE=2: every PCM list on the pipelined kernel (A/B)
    int lanes = kLanes;                                 // WVG_LANES: streams per decode (A/B of the queue mapping)
    bool lanes_env = false;                             // WVG_LANES given: no in-flight policy (wvg_batch_decode)
    int lane_mode = 1;                                  // term-set groups on the lane-per-block kernel (wvg_batch_set_kernel)
    uint32_t lane_groups = 0;                           // the last decode's groups on lane kernels (wvg_batch_lane_groups)
    bool kernel_auto = true;                            // WVG_KERNEL_AUTO: lane_mode chosen per decode and group
    bool log_decodes = false;                           // WVG_DECODE_LOG=1: each decode's streams and kernels on stderr
    std::vector<uint32_t> h_status, h_aux;
    int64_t bytes_in = 0, frames = 0;
    // format epilogue: per-file byte image of WavpackFormatSamples
    std::vector<int64_t> pcm_off;                       // per file, -1 when it did not open
    int64_t pcm_bytes = 0;
    std::vector<FormatSeg> segs;
    // device
    uint8_t *d_blob = nullptr, *d_tables = nullptr, *d_pcm = nullptr;
    BlockDesc *d_descs = nullptr;
    MetaItem *d_items = nullptr;  // deferred metadata values (wv_meta.h), applied once per upload
    MetaJob *d_jobs = nullptr;
    FormatSeg *d_segs = nullptr;
    ZeroSeg *d_zeros = nullptr;  // the framing's gap zero-fills (FramingOutput::zeros), written by each decode
    size_t cap_zeros = 0;
    uint32_t nzeros = 0;
    int32_t *d_out = nullptr;
    uint32_t *d_status = nullptr, *d_mute = nullptr, *d_pcml = nullptr, *d_dsd = nullptr;
    bool uploaded = false, downloaded = false, formatted = false;
    // device-side framing (wv_dframe.h): files added by wvg_batch_add_files_device
    // are framed at upload, on the device, or by the host when outside its scope
    struct PendingFile {
        size_t base, len;
        int idx;
    };
    std::vector<PendingFile> dfiles;
    int64_t framed_dev = 0, framed_host = 0;
    PinnedBuf dfst;  // page-locked staging of the framing passes
    DFile *d_dfiles = nullptr;
    uint64_t *d_slots = nullptr;
    uint32_t *d_blkf = nullptr, *d_blkk = nullptr, *d_tfile = nullptr, *d_rankf = nullptr, *d_cand = nullptr,
             *d_cnt = nullptr;
    size_t cap_tfile = 0, cap_rankf = 0, cap_cand = 0, cap_cnt = 0;
    int64_t rank_min = 256 * 1024;  // files from this size on take the parallel header walk (WVG_DFRAME_RANK_MIN)
    BlockDesc *d_ddescs = nullptr;
    DBlock *d_drecs = nullptr;
    // descriptors the device framing left in d_ddescs: descriptors [dst, dst + n)
    // of the batch are d_ddescs[src, src + n) (the host keeps only their head,
    // kDescHead bytes); the upload copies them into d_descs on the device
    struct DevRun {
        size_t dst, src, n;
    };
    std::vector<DevRun> dev_runs;
    size_t cap_dfiles = 0, cap_slots = 0, cap_blkf = 0, cap_blkk = 0, cap_ddescs = 0, cap_drecs = 0;
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

// grow-only device allocation: a batch that is refilled and re-uploaded keeps its buffers
template <class T>
static hipError_t ensure(T *&p, size_t &cap, size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
}

extern "C" {

wvg_ctx *wvg_open(int device) {
    // A decode launches one kernel group per stream (term sets, generic PCM, DSD,
    // DSD mode 1) and keeps several batches in flight; HIP's default of 4 hardware
    // queues per process makes streams share queues, and a queue runs its kernels
    // one after another (a mixed batch then waits for its DSD mode-3 chains before
    // the PCM groups queued behind them).  The queue count is the host's choice
    // (GPU_MAX_HW_QUEUES before the process's first HIP call): the
    // library never changes the process environment.
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return nullptr;
    if (device < 0) hipGetDevice(&device);
    if (device >= n || hipSetDevice(device) != hipSuccess) return nullptr;
    if (upload_dsd_ptables() != hipSuccess) return nullptr;  // DSD mode 3's starting tables, per device
    wvg_ctx *c = new wvg_ctx();
    c->device = device;
    const char *q = getenv("GPU_MAX_HW_QUEUES");
    if (q && atoi(q) >= 1) c->hw_queues = atoi(q);
    const char *ds = getenv("WVG_DSD_STREAM");
    if (ds && (ds[0] == '0' || ds[0] == '1')) c->own_streams = ds[0] - '0';
    return c;
}

void wvg_close(wvg_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    for (hipStream_t &st : c->side)
        if (st) {
            hipStreamSynchronize(st);
            hipStreamDestroy(st);
        }
    delete c;
}

const char *wvg_last_error(wvg_ctx *c) { return c ? c->err.c_str() : "no context"; }

static void free_streams(wvg_batch *b) {
    for (int i = 0; i < kLanes - 1; i++)
        if (b->join[i]) hipEventDestroy(b->join[i]);
    if (b->fork) hipEventDestroy(b->fork);
    if (b->done) hipEventDestroy(b->done);
    if (b->up) hipEventDestroy(b->up);
    if (b->stream) hipStreamDestroy(b->stream);
    for (hipStream_t &d : b->dstream)
        if (d) hipStreamDestroy(d);
    for (auto &e : b->tev) hipEventDestroy(e);
    for (auto &e : b->tfree) hipEventDestroy(e);
    b->tev.clear();
    b->tfree.clear();
    for (auto &e : b->gev)
        if (e) hipEventDestroy(e);
}

wvg_batch *wvg_batch_new(wvg_ctx *c, int chunk_frames) {
    if (!c || chunk_frames <= 0) return nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return nullptr;
    wvg_batch *b = new wvg_batch();
    b->ctx = c;
    b->chunk = chunk_frames;
    // side streams are created on first use (a batch with one launch group needs
    // none): every stream takes one of the process's few hardware queues
    // (GPU_MAX_HW_QUEUES), and batches in flight should each get their own
    bool ok = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&b->fork, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&b->done, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&b->up, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        free_streams(b);
        delete b;
        return nullptr;
    }
    const char *fl = getenv("WVG_FORCE_LANE");
    b->force_lane = fl && fl[0] == '1';
    const char *pp = getenv("WVG_PIPE");
    b->prefer_pipe = pp ? atoi(pp) : 0;
    // the decorr/entropy values of each block are parsed on the device (wv_meta_parse);
    // WVG_HOST_META=1 keeps them on the host framing (A/B comparisons)
    const char *ln = getenv("WVG_LANES");
    if (ln && atoi(ln) >= 1) {
        b->lanes = atoi(ln) < kLanes ? atoi(ln) : kLanes;
        b->lanes_env = true;
    }
    const char *lk = getenv("WVG_LANE_KERNEL");
    b->lane_mode = lk ? atoi(lk) : 1;  // (default: WVG_KERNEL_AUTO, wvg_batch_set_kernel)
    b->kernel_auto = !lk;
    const char *dl = getenv("WVG_DECODE_LOG");
    b->log_decodes = dl && dl[0] == '1';
    const char *rm = getenv("WVG_DFRAME_RANK_MIN");
    if (rm) b->rank_min = atoll(rm);
    const char *hm = getenv("WVG_HOST_META");
    b->fo.defer_values = !(hm && hm[0] == '1');
    const char *lc = getenv("WVG_LANE_COUNTERS");
    if (lc && lc[0] == '1') {
        const size_t bytes = sizeof(uint32_t) * 16u * kLaneDbgWaves * kMaxTermSets;
        if (hipMalloc(&b->d_lane_dbg, bytes) != hipSuccess || hipMemset(b->d_lane_dbg, 0, bytes) != hipSuccess)
            b->d_lane_dbg = nullptr;
    }
    {
        std::lock_guard<std::mutex> g(c->mu);
        c->batches.push_back(b);
    }
    return b;
}

static void free_dev(wvg_batch *b) {
    hipFree(b->d_blob);
    hipFree(b->d_lane_dbg);
    b->d_lane_dbg = nullptr;
    hipFree(b->d_tables);
    hipFree(b->d_pcm);
    hipFree(b->d_descs);
    hipFree(b->d_items);
    hipFree(b->d_jobs);
    hipFree(b->d_segs);
    hipFree(b->d_zeros);
    hipFree(b->d_out);
    hipFree(b->d_status);
    hipFree(b->d_mute);
    hipFree(b->d_pcml);
    hipFree(b->d_dsd);
    hipFree(b->d_dfiles);
    hipFree(b->d_slots);
    hipFree(b->d_blkf);
    hipFree(b->d_blkk);
    hipFree(b->d_tfile);
    hipFree(b->d_rankf);
    hipFree(b->d_cand);
    hipFree(b->d_cnt);
    b->d_tfile = b->d_rankf = b->d_cand = b->d_cnt = nullptr;
    b->cap_tfile = b->cap_rankf = b->cap_cand = b->cap_cnt = 0;
    hipFree(b->d_ddescs);
    hipFree(b->d_drecs);
    b->d_dfiles = nullptr;
    b->d_slots = nullptr;
    b->d_blkf = b->d_blkk = nullptr;
    b->d_ddescs = nullptr;
    b->d_drecs = nullptr;
    b->cap_dfiles = b->cap_slots = b->cap_blkf = b->cap_blkk = b->cap_ddescs = b->cap_drecs = 0;
    for (int t = 0; t < kMaxTermSets; t++) {
        hipFree(b->d_ts[t]);
        b->d_ts[t] = nullptr;
        b->cap_ts[t] = 0;
    }
    b->d_blob = b->d_tables = b->d_pcm = nullptr;
    b->d_descs = nullptr;
    b->d_items = nullptr;
    b->d_jobs = nullptr;
    b->d_segs = nullptr;
    b->d_zeros = nullptr;
    b->cap_zeros = 0;
    b->d_out = nullptr;
    b->d_status = b->d_mute = b->d_pcml = b->d_dsd = nullptr;
    b->cap_blob = b->cap_descs = b->cap_items = b->cap_jobs = b->cap_tables = b->cap_out = b->cap_st = 0;
    b->cap_pcml = b->cap_dsd = b->cap_pcm = b->cap_segs = 0;
    b->uploaded = b->formatted = b->segs_uploaded = false;
}

// Wait for everything that may still read or write the batch's device buffers:
// its own stream, and the last decode/format, which may have run on a caller's
// stream (`done` is recorded there).  The buffers are grow-only and reused, so
// a reset/re-upload must not overwrite them under a running kernel.
static hipError_t quiesce(wvg_batch *b) {
    hipError_t e = hipSuccess;
    if (b->done) e = hipEventSynchronize(b->done);
    if (b->stream) {
        hipError_t e2 = hipStreamSynchronize(b->stream);
        if (e == hipSuccess) e = e2;
    }
    return e;
}

// Grow the page-locked blob: a larger one is a new allocation, so a DMA still
// reading the old one must finish first.
static bool blob_resize(wvg_batch *b, size_t n) {
    if (n > b->blob.cap && b->blob_dma) {
        hipStreamSynchronize(b->stream);
        b->blob_dma = false;
    }
    return b->blob.resize(n);
}

// Send the blob bytes copied in since the last push (on the batch stream, ahead
// of the framing kernels and decodes that read them): the DMA of files added
// early overlaps the copying and framing of the rest.  A d_blob too small for
// them is replaced (after anything in flight that reads it) and refilled whole.
static hipError_t blob_push(wvg_batch *b, size_t upto = (size_t)-1) {
    // a decode of the earlier files (on a caller's stream) may still read past their
    // end, where new bytes now land
    if (b->done) {
        hipError_t e = hipEventSynchronize(b->done);
        if (e != hipSuccess) return e;
    }
    const size_t need = b->blob.size() + 64;  // the whole blob and the reader's 0xFF tail
    if (b->cap_blob < need) {
        hipError_t e = quiesce(b);
        if (e != hipSuccess) return e;
        e = ensure(b->d_blob, b->cap_blob, b->cap_blob * 2 > need ? b->cap_blob * 2 : need);
        if (e != hipSuccess) return e;
        b->blob_dev = 0;
    }
    const size_t n = upto < b->blob.size() ? upto : b->blob.size();
    if (n <= b->blob_dev) return hipSuccess;
    hipError_t e = hipMemcpyAsync(b->d_blob + b->blob_dev, b->blob.data() + b->blob_dev, n - b->blob_dev,
                                  hipMemcpyHostToDevice, b->stream);
    if (e != hipSuccess) return e;
    b->blob_dev = n;
    b->blob_dma = true;
    return hipSuccess;
}

void wvg_batch_free(wvg_batch *b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->ctx->mu);
        auto &v = b->ctx->batches;
        v.erase(std::remove(v.begin(), v.end(), b), v.end());
    }
    hipSetDevice(b->ctx->device);
    quiesce(b);
    free_dev(b);
    free_streams(b);
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
    wi.seek_result = fi.seek_result;
    wi.sample_index0 = fi.sample_index0;
}

int wvg_probe_file(const uint8_t *file, size_t len, uint32_t open_flags, int chunk_frames, wvg_file_info *info) {
    if ((!file && len) || !info) return WVG_ERR_ARG;
    FramingOutput fo;
    FileInfo fi;
    frame_file(file, len, 0, 0, open_flags, chunk_frames > 0 ? chunk_frames : 4096, fo, fi);
    fill_info(fi, *info);
    return fi.open_ok ? WVG_OK : WVG_ERR_OPEN;
}

// Record a framed file in the batch: the getters' view, its output range, its
// WavpackFormatSamples segments and its blocks' launch groups.  `fi` refers to
// descriptors already in b->fo.
// `at` >= 0: the file's slot was reserved when it was added (device framing).
static int commit_file(wvg_batch *b, FileInfo &fin, size_t len, wvg_file_info *info, int at = -1) {
    wvg_file_info wi;
    fill_info(fin, wi);
    wi.out_offset = b->out_ints;
    wi.header_off = fin.header_off;
    wi.header_len = fin.header_len;
    wi.trailer_off = fin.trailer_off;
    wi.trailer_len = fin.trailer_len;
    // (the FileInfo moves into the batch: its call cuts and error text are not copied)
    if (at < 0) {
        at = (int)b->infos.size();
        b->finfo.push_back(std::move(fin));
        b->infos.push_back(wi);
        b->pcm_off.push_back(-1);
    } else {
        b->finfo[(size_t)at] = std::move(fin);
        b->infos[(size_t)at] = wi;
    }
    const FileInfo &fi = b->finfo[(size_t)at];
    if (info) *info = wi;
    if (!fi.open_ok) return WVG_ERR_OPEN;
    // the file's WavpackFormatSamples image: frames x reduced channels x bytes per sample, 16-B aligned
    const int64_t nvals = fi.out_frames * fi.out_nch;
    b->pcm_bytes = (b->pcm_bytes + 15) & ~(int64_t)15;
    b->pcm_off[(size_t)at] = b->pcm_bytes;
    for (int64_t s = 0; s < nvals; s += kFormatSeg) {
        FormatSeg g;
        g.in_off = (uint64_t)(b->out_ints + s);
        g.out_off = (uint64_t)(b->pcm_bytes + s * wi.bytes_per_sample);
        g.n = (uint32_t)(nvals - s < (int64_t)kFormatSeg ? nvals - s : kFormatSeg);
        g.bps = (uint32_t)wi.bytes_per_sample;
        b->segs.push_back(g);
    }
    b->pcm_bytes += nvals * wi.bytes_per_sample;
    // the output range reserved for the file covers every descriptor's writes
    const int64_t extent = file_out_extent(b->fo, fi, (uint64_t)b->out_ints);
    b->out_ints += extent;
    for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++) {
        const BlockDesc &d = b->fo.descs[(size_t)k];
        b->frames += d.nframes;
        // a chain member is decoded by its chain's first block (wv_decode_pcm_wave /
        // wv_decode_dsd_wave); DSD members stay in the DSD list for the mute fills (wv_dsd_fill)
        if ((d.inherit & INH_MEMBER) && d.kind == KIND_PCM) continue;
        int ts = (d.kind == KIND_PCM && !b->force_lane) ? term_set_of(d, b->prefer_pipe) : -1;
        if (ts >= 0) b->ts_list[ts].push_back((uint32_t)k);
        else if (d.kind == KIND_PCM) b->pcm_list.push_back((uint32_t)k);
        else if (d.kind != KIND_SKIP) b->dsd_list.push_back((uint32_t)k);
    }
    // compressed bytes of the file's decoded blocks (whole file is a fine proxy)
    b->bytes_in += (int64_t)len;
    return at;
}

static int add_file(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, int64_t seek_to,
                    wvg_file_info *info) {
    if (!b || (!file && len)) return WVG_ERR_ARG;
    b->uploaded = b->formatted = false;
    size_t base = (b->blob.size() + 15) & ~(size_t)15;
    if (!blob_resize(b, base + len)) {
        b->ctx->err = "out of host memory";
        return WVG_ERR_ARG;
    }
    if (len) memcpy(b->blob.data() + base, file, len);
    FileInfo fi;
    b->fo.chain_tables_only = true;  // (the device builds every unchained mode-1 block's tables)
    frame_file(b->blob.data() + base, len, base, (uint64_t)b->out_ints, open_flags, b->chunk, b->fo, fi, seek_to);
    return commit_file(b, fi, len, info);
}

int wvg_batch_reset(wvg_batch *b) {
    if (!b) return WVG_ERR_ARG;
    hipSetDevice(b->ctx->device);
    quiesce(b);  // nothing in flight reads the old contents (on the batch's or a caller's stream)
    b->blob.resize(0);
    b->blob_dev = 0;
    b->blob_dma = false;
    const bool defer = b->fo.defer_values;
    b->fo = FramingOutput();
    b->fo.defer_values = defer;
    b->finfo.clear();
    b->infos.clear();
    b->out_ints = 0;
    b->pcm_list.clear();
    b->dsd_list.clear();
    for (auto &l : b->ts_list) l.clear();
    b->h_status.clear();
    b->h_aux.clear();
    b->bytes_in = b->frames = 0;
    b->pcm_off.clear();
    b->pcm_bytes = 0;
    b->segs.clear();
    b->uploaded = b->downloaded = b->formatted = b->segs_uploaded = false;
    b->dfiles.clear();
    b->dev_runs.clear();
    b->framed_dev = b->framed_host = 0;
    return WVG_OK;
}

int wvg_batch_add_file(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, wvg_file_info *info) {
    return add_file(b, file, len, open_flags, -1, info);
}

// Frame files already in the blob on host threads, each into its own
// FramingOutput with out offsets relative to 0 (merge_framed moves them).
static void frame_threaded(wvg_batch *b, const std::vector<size_t> &base, const std::vector<size_t> &lens,
                           uint32_t open_flags, int threads, std::vector<FramingOutput> &fos,
                           std::vector<FileInfo> &fis) {
    const int n = (int)base.size();
    if (threads <= 0) {
        const char *e = getenv("WVG_FRAME_THREADS");
        threads = e ? atoi(e) : (int)std::thread::hardware_concurrency();
        if (threads > 16) threads = 16;  // the lease's CPU share on the GPU boxes
    }
    if (threads < 1) threads = 1;
    if (threads > n) threads = n > 0 ? n : 1;
    fos.assign((size_t)n, FramingOutput());
    fis.assign((size_t)n, FileInfo());
    for (auto &f : fos) {
        f.defer_values = b->fo.defer_values;
        f.chain_tables_only = true;  // (the device builds every unchained mode-1 block's tables)
    }
    std::atomic<int> next(0);
    auto work = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;)
            frame_file(b->blob.data() + base[(size_t)i], lens[(size_t)i], base[(size_t)i], 0, open_flags, b->chunk,
                       fos[(size_t)i], fis[(size_t)i], -1);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
}

// The files' bytes into the page-locked blob on host threads, in pieces of up to 4 MiB
// (one thread copies a 53 MB file at ~15 GB/s: 3.4 ms of a C2 request's host time, and a
// 12,500-file C5 slice's 540 MB took ~50 of its ~70 ms of framing)
static double now_ms();

static void parallel_copy(uint8_t *blob, const uint8_t *const *files, const size_t *lens,
                          const std::vector<size_t> &base, int n, int threads) {
    constexpr size_t kPiece = (size_t)4 << 20;
    struct Piece {
        uint8_t *dst;
        const uint8_t *src;
        size_t len;
    };
    std::vector<Piece> pieces;
    size_t total = 0;
    for (int i = 0; i < n; i++) {
        for (size_t o = 0; o < lens[i]; o += kPiece)
            pieces.push_back({blob + base[(size_t)i] + o, files[i] + o, std::min(kPiece, lens[i] - o)});
        total += lens[i];
    }
    if (threads <= 0) {
        const char *e = getenv("WVG_FRAME_THREADS");
        threads = e ? atoi(e) : (int)std::thread::hardware_concurrency();
        if (threads > 16) threads = 16;  // the lease's CPU share on the GPU boxes
    }
    const size_t want = total / kPiece + 1;  // (one thread per piece at most)
    if ((size_t)threads > want) threads = (int)want;
    if (threads < 1) threads = 1;
    std::atomic<size_t> next(0);
    auto work = [&]() {
        for (size_t k; (k = next.fetch_add(1)) < pieces.size();) memcpy(pieces[k].dst, pieces[k].src, pieces[k].len);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
}

// Append one file framed by frame_threaded to the batch at the current output
// end and commit it (at: its reserved file slot, or -1 for a new one).
static int merge_framed(wvg_batch *b, FramingOutput &f, FileInfo &fi, size_t len, wvg_file_info *info, int at) {
    const uint64_t ob = (uint64_t)b->out_ints;
    const uint32_t d0 = (uint32_t)b->fo.descs.size(), i0 = (uint32_t)b->fo.items.size();
    const size_t t0 = (b->fo.tables.size() + 15) & ~(size_t)15;
    for (BlockDesc &d : f.descs) {
        d.out_off += ob;  // wrapping add: a seek's offsets may lie before the file's output
        d.dsd_table_off += t0;
    }
    for (MetaJob &j : f.jobs) {
        j.desc += d0;
        j.first += i0;
    }
    b->fo.descs.insert(b->fo.descs.end(), f.descs.begin(), f.descs.end());
    b->fo.items.insert(b->fo.items.end(), f.items.begin(), f.items.end());
    b->fo.jobs.insert(b->fo.jobs.end(), f.jobs.begin(), f.jobs.end());
    if (!f.tables.empty()) {
        b->fo.tables.resize(t0);
        b->fo.tables.insert(b->fo.tables.end(), f.tables.begin(), f.tables.end());
    }
    for (ZeroSeg z : f.zeros) {
        z.off += ob;
        b->fo.zeros.push_back(z);
    }
    fi.first_desc += d0;
    return commit_file(b, fi, len, info, at);
}

// Many files at once: the bytes are copied into the blob, the files are framed
// on host threads (each into its own FramingOutput, out offsets relative to 0),
// then merged in file order with their offsets moved to the batch's.
int wvg_batch_add_files(wvg_batch *b, int n, const uint8_t *const *files, const size_t *lens, uint32_t open_flags,
                        int threads, wvg_file_info *infos, int32_t *indices) {
    if (!b || n < 0 || (n && (!files || !lens))) return WVG_ERR_ARG;
    b->uploaded = b->formatted = false;
    std::vector<size_t> base((size_t)n);
    size_t end = b->blob.size();
    for (int i = 0; i < n; i++) {
        if (!files[i] && lens[i]) return WVG_ERR_ARG;
        base[(size_t)i] = (end + 15) & ~(size_t)15;
        end = base[(size_t)i] + lens[i];
    }
    if (!blob_resize(b, end)) {
        b->ctx->err = "out of host memory";
        return WVG_ERR_ARG;
    }
    static const bool trace = getenv("WVG_ADD_TRACE") && getenv("WVG_ADD_TRACE")[0] == '1';
    const double t0 = trace ? now_ms() : 0.0;
    parallel_copy(b->blob.data(), files, lens, base, n, threads);
    const double t1 = trace ? now_ms() : 0.0;
    HIPCHK(b->ctx, hipSetDevice(b->ctx->device));
    HIPCHK(b->ctx, blob_push(b));  // the DMA runs while the host threads frame the files
    std::vector<size_t> ln(lens, lens + n);
    std::vector<FramingOutput> fos;
    std::vector<FileInfo> fis;
    const double t2 = trace ? now_ms() : 0.0;
    frame_threaded(b, base, ln, open_flags, threads, fos, fis);
    const double t3 = trace ? now_ms() : 0.0;
    {   // (the merge appends every file's records: one allocation each, not a doubling series)
        size_t nd = b->fo.descs.size(), ni = b->fo.items.size(), nj = b->fo.jobs.size(), nz = b->fo.zeros.size();
        for (const FramingOutput &f : fos) {
            nd += f.descs.size();
            ni += f.items.size();
            nj += f.jobs.size();
            nz += f.zeros.size();
        }
        b->fo.descs.reserve(nd);
        b->fo.items.reserve(ni);
        b->fo.jobs.reserve(nj);
        b->fo.zeros.reserve(nz);
        const size_t nf = b->finfo.size() + (size_t)n;
        b->finfo.reserve(nf);
        b->infos.reserve(nf);
        b->pcm_off.reserve(nf);
    }
    for (int i = 0; i < n; i++) {
        const int idx = merge_framed(b, fos[(size_t)i], fis[(size_t)i], lens[i], infos ? &infos[i] : nullptr, -1);
        if (indices) indices[i] = idx;
    }
    if (trace)
        fprintf(stderr, "wvg add_files: %d files, copy %.2f ms, push %.2f, frame %.2f, merge %.2f\n", n, t1 - t0,
                t2 - t1, t3 - t2, now_ms() - t3);
    return n;
}

// A hybrid file with its .wvc correction file (beyond the reference, which
// never reads the correction stream: SURVEY §8f-4): both are copied into the blob
// and the hybrid blocks decode exactly.
int wvg_batch_add_file_wvc(wvg_batch *b, const uint8_t *file, size_t len, const uint8_t *wvc, size_t wvc_len,
                           uint32_t open_flags, wvg_file_info *info) {
    if (!b || (!file && len) || (!wvc && wvc_len)) return WVG_ERR_ARG;
    b->uploaded = b->formatted = false;
    const size_t base = (b->blob.size() + 15) & ~(size_t)15;
    const size_t cbase = (base + len + 15) & ~(size_t)15;
    if (!blob_resize(b, cbase + wvc_len)) {
        b->ctx->err = "out of host memory";
        return WVG_ERR_ARG;
    }
    if (len) memcpy(b->blob.data() + base, file, len);
    if (wvc_len) memcpy(b->blob.data() + cbase, wvc, wvc_len);
    FileInfo fi;
    b->fo.chain_tables_only = true;
    frame_file(b->blob.data() + base, len, base, (uint64_t)b->out_ints, open_flags, b->chunk, b->fo, fi, -1,
               wvc_len ? b->blob.data() + cbase : nullptr, wvc_len, cbase);
    return commit_file(b, fi, len + wvc_len, info);
}

int wvg_batch_add_file_at(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, int64_t start_sample,
                          wvg_file_info *info) {
    if (start_sample < 0) return WVG_ERR_ARG;
    return add_file(b, file, len, open_flags, start_sample, info);
}

// Files whose framing waits for the upload: their bytes are copied into the
// blob and their file slots reserved; wvg_batch_upload frames them on the device
// (wv_dframe.h), or on the host when a file is outside the device scope.
int wvg_batch_add_files_device(wvg_batch *b, int n, const uint8_t *const *files, const size_t *lens,
                               int32_t *indices) {
    if (!b || n < 0 || (n && (!files || !lens))) return WVG_ERR_ARG;
    b->uploaded = b->formatted = false;
    size_t end = b->blob.size();
    std::vector<size_t> base((size_t)n);
    for (int i = 0; i < n; i++) {
        if (!files[i] && lens[i]) return WVG_ERR_ARG;
        base[(size_t)i] = (end + 15) & ~(size_t)15;
        end = base[(size_t)i] + lens[i];
    }
    if (!blob_resize(b, end)) {
        b->ctx->err = "out of host memory";
        return WVG_ERR_ARG;
    }
    HIPCHK(b->ctx, hipSetDevice(b->ctx->device));
    // the bytes on host threads (parallel_copy), then one DMA of them: a 12,500-file C5 slice's
    // 540 MB took 36 ms on this thread, piece by piece behind the pushes
    parallel_copy(b->blob.data(), files, lens, base, n, 0);
    HIPCHK(b->ctx, blob_push(b));
    FileInfo fi0;
    fi0.error = "not framed yet (wvg_batch_upload frames it)";
    wvg_file_info wi;
    fill_info(fi0, wi);
    const size_t nf = b->finfo.size() + (size_t)n;
    b->finfo.reserve(nf);
    b->infos.reserve(nf);
    b->pcm_off.reserve(nf);
    b->dfiles.reserve(b->dfiles.size() + (size_t)n);
    for (int i = 0; i < n; i++) {
        const int idx = (int)b->infos.size();
        b->finfo.push_back(fi0);
        b->infos.push_back(wi);
        b->pcm_off.push_back(-1);
        b->dfiles.push_back({base[(size_t)i], lens[i], idx});
        if (indices) indices[i] = idx;
    }
    return n;
}

// The framing passes of the pending files (the blob is on the device already):
// the walk (one lane per file), the output range of every file it accepted, the
// block pass (one lane per block), then, in file order, the accepted files'
// descriptors committed and every other file framed by the host.
// WVG_DFRAME_TRACE=1 (diagnostic): the host-side phases of each device framing on stderr
static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int device_frame(wvg_batch *b, hipStream_t s) {
    wvg_ctx *c = b->ctx;
    static const bool trace = getenv("WVG_DFRAME_TRACE") && getenv("WVG_DFRAME_TRACE")[0] == '1';
    double tp[6] = {now_ms(), 0, 0, 0, 0, 0};
    const size_t nf = b->dfiles.size();
    std::vector<DFile> df(nf);
    uint64_t nslots = 0;
    // large files: the parallel header walk (candidate scan over 8 KiB tiles + list ranking)
    std::vector<uint32_t> tfile, rankf;
    const size_t tb = dframe_tile_bytes();
    for (size_t i = 0; i < nf; i++) {
        memset(&df[i], 0, sizeof(DFile));
        df[i].base = b->dfiles[i].base;
        df[i].len = b->dfiles[i].len;
        df[i].slot = nslots;
        df[i].chunk = (uint32_t)b->chunk;
        nslots += b->dfiles[i].len / 32 + 1;
        if (b->rank_min >= 0 && (int64_t)df[i].len >= b->rank_min && df[i].len >= 32) {
            df[i].tile0 = (uint32_t)tfile.size();
            df[i].ntiles = (uint32_t)((df[i].len + tb - 1) / tb);
            tfile.insert(tfile.end(), df[i].ntiles, (uint32_t)i);
            rankf.push_back((uint32_t)i);
        }
    }
    HIPCHK(c, ensure(b->d_dfiles, b->cap_dfiles, sizeof(DFile) * (nf ? nf : 1)));
    HIPCHK(c, ensure(b->d_slots, b->cap_slots, sizeof(uint64_t) * (nslots ? nslots : 1)));
    const size_t nt = tfile.size(), nr = rankf.size();
    if (!b->dfst.resize(sizeof(DFile) * nf + sizeof(uint32_t) * (nt + nr))) return WVG_ERR_SPACE;
    memcpy(b->dfst.data(), df.data(), sizeof(DFile) * nf);
    HIPCHK(c, hipMemcpyAsync(b->d_dfiles, b->dfst.data(), sizeof(DFile) * nf, hipMemcpyHostToDevice, s));
    if (nr) {
        uint32_t *h = reinterpret_cast<uint32_t *>(b->dfst.data() + sizeof(DFile) * nf);
        memcpy(h, tfile.data(), sizeof(uint32_t) * nt);
        memcpy(h + nt, rankf.data(), sizeof(uint32_t) * nr);
        HIPCHK(c, ensure(b->d_tfile, b->cap_tfile, sizeof(uint32_t) * nt));
        HIPCHK(c, ensure(b->d_rankf, b->cap_rankf, sizeof(uint32_t) * nr));
        const size_t ncand = nt * dframe_tile_cap() + 1024;
        HIPCHK(c, ensure(b->d_cand, b->cap_cand, sizeof(uint32_t) * ncand));
        HIPCHK(c, ensure(b->d_cnt, b->cap_cnt, sizeof(uint32_t) * (2 * nt + 1)));
        HIPCHK(c, hipMemcpyAsync(b->d_tfile, h, sizeof(uint32_t) * nt, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(b->d_rankf, h + nt, sizeof(uint32_t) * nr, hipMemcpyHostToDevice, s));
        HIPCHK(c, launch_dframe_rank(b->d_dfiles, b->d_tfile, (uint32_t)nt, b->d_rankf, (uint32_t)nr, b->d_blob,
                                     b->d_cand, (uint32_t)ncand, b->d_cnt, b->d_slots, s));
    }
    HIPCHK(c, launch_dframe_walk(b->d_dfiles, (uint32_t)nf, b->d_blob, b->d_slots, s));
    HIPCHK(c, hipMemcpyAsync(b->dfst.data(), b->d_dfiles, sizeof(DFile) * nf, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    tp[1] = now_ms();
    memcpy(df.data(), b->dfst.data(), sizeof(DFile) * nf);
    // output ranges and the block list of the accepted files, in file order
    std::vector<uint32_t> bf, bk;
    std::vector<size_t> blk0(nf, 0);
    int64_t ob = b->out_ints;
    for (size_t i = 0; i < nf; i++) {
        if (!df[i].regular) continue;
        df[i].out_base = (uint64_t)ob;
        blk0[i] = bf.size();
        for (uint32_t k = 0; k < df[i].nblocks; k++) {
            bf.push_back((uint32_t)i);
            bk.push_back(k);
        }
        ob += df[i].total_samples * df[i].nch;
    }
    const size_t nb = bf.size();
    std::vector<DBlock> recs(nb);
    const uint8_t *heads = nullptr;  // each device descriptor's first kDescHead bytes (staging)
    if (nb && !b->dev_runs.empty()) {
        // an earlier device framing of this batch left descriptors in d_ddescs, which
        // this pass reuses: bring them to the host first (files added after an upload
        // without a reset -- not the common path)
        for (const auto &r : b->dev_runs)
            HIPCHK(c, hipMemcpyAsync(b->fo.descs.data() + r.dst, b->d_ddescs + r.src, sizeof(BlockDesc) * r.n,
                                     hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        b->dev_runs.clear();
    }
    if (nb) {
        HIPCHK(c, ensure(b->d_blkf, b->cap_blkf, sizeof(uint32_t) * nb));
        HIPCHK(c, ensure(b->d_blkk, b->cap_blkk, sizeof(uint32_t) * nb));
        HIPCHK(c, ensure(b->d_ddescs, b->cap_ddescs, sizeof(BlockDesc) * nb));
        HIPCHK(c, ensure(b->d_drecs, b->cap_drecs, sizeof(DBlock) * nb));
        // up and down in separate parts of the staging: no wait between the copies and the pass
        const size_t up = sizeof(DFile) * nf + 2 * sizeof(uint32_t) * nb;
        const size_t up_al = (up + 255) & ~(size_t)255;
        const size_t down = (kDescHead + sizeof(DBlock)) * nb;
        if (!b->dfst.resize(up_al + down)) return WVG_ERR_SPACE;
        uint8_t *h = b->dfst.data();
        memcpy(h, df.data(), sizeof(DFile) * nf);
        memcpy(h + sizeof(DFile) * nf, bf.data(), sizeof(uint32_t) * nb);
        memcpy(h + sizeof(DFile) * nf + sizeof(uint32_t) * nb, bk.data(), sizeof(uint32_t) * nb);
        HIPCHK(c, hipMemcpyAsync(b->d_dfiles, h, sizeof(DFile) * nf, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(b->d_blkf, h + sizeof(DFile) * nf, sizeof(uint32_t) * nb, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(b->d_blkk, h + sizeof(DFile) * nf + sizeof(uint32_t) * nb, sizeof(uint32_t) * nb,
                                 hipMemcpyHostToDevice, s));
        tp[2] = now_ms();
        HIPCHK(c, launch_dframe_block(b->d_dfiles, b->d_blkf, b->d_blkk, (uint32_t)nb, b->d_blob, b->d_slots,
                                      b->d_ddescs, b->d_drecs, s));
        // the descriptors stay on the device; the host takes each one's head (a strided
        // copy) and the per-block records it reduces into the FileInfo
        uint8_t *hd = h + up_al;
        HIPCHK(c, hipMemcpy2DAsync(hd, kDescHead, b->d_ddescs, sizeof(BlockDesc), kDescHead, nb, hipMemcpyDeviceToHost,
                                   s));
        HIPCHK(c, hipMemcpyAsync(hd + kDescHead * nb, b->d_drecs, sizeof(DBlock) * nb, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        tp[3] = now_ms();
        heads = hd;
        memcpy(recs.data(), hd + kDescHead * nb, sizeof(DBlock) * nb);
    }
    b->fo.descs.reserve(b->fo.descs.size() + nb);
    // commit: the accepted files at their reserved output ranges, in file order
    std::vector<size_t> host;
    for (size_t i = 0; i < nf; i++) {
        const auto &p = b->dfiles[i];
        FileInfo fi;
        fi.blob_base = p.base;
        fi.first_desc = (int64_t)b->fo.descs.size();
        if (df[i].regular && dframe_file_info(df[i], recs.data() + blk0[i], fi)) {
            const size_t dst = b->fo.descs.size();
            b->fo.descs.resize(dst + df[i].nblocks);  // zeroed; the host's view is each head
            for (uint32_t k = 0; k < df[i].nblocks; k++)
                memcpy(&b->fo.descs[dst + k], heads + kDescHead * (blk0[i] + k), kDescHead);
            if (!b->dev_runs.empty() && b->dev_runs.back().dst + b->dev_runs.back().n == dst &&
                b->dev_runs.back().src + b->dev_runs.back().n == blk0[i])
                b->dev_runs.back().n += df[i].nblocks;  // contiguous with the previous file's
            else
                b->dev_runs.push_back({dst, blk0[i], (size_t)df[i].nblocks});
            b->out_ints = (int64_t)df[i].out_base;
            commit_file(b, fi, p.len, nullptr, p.idx);
            b->framed_dev++;
        } else {
            host.push_back(i);
        }
    }
    if (b->out_ints < ob) b->out_ints = ob;  // a range whose file fell back to the host stays unused
    if (!host.empty()) {  // the host framing of the rest, on host threads
        std::vector<size_t> hb, hl;
        for (size_t i : host) {
            hb.push_back(b->dfiles[i].base);
            hl.push_back(b->dfiles[i].len);
        }
        std::vector<FramingOutput> fos;
        std::vector<FileInfo> fis;
        frame_threaded(b, hb, hl, 0, 0, fos, fis);
        for (size_t j = 0; j < host.size(); j++) {
            merge_framed(b, fos[j], fis[j], hl[j], nullptr, b->dfiles[host[j]].idx);
            b->framed_host++;
        }
    }
    b->dfiles.clear();
    if (trace) {
        tp[4] = now_ms();
        fprintf(stderr, "dframe: walk+sync %.3f  lists+sync %.3f  block+D2H %.3f  commit+host %.3f ms (%zu files)\n",
                tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], nf);
    }
    return WVG_OK;
}

int wvg_batch_file_info(const wvg_batch *b, int file, wvg_file_info *info) {
    if (!b || !info || file < 0 || file >= (int)b->infos.size()) return WVG_ERR_ARG;
    *info = b->infos[(size_t)file];
    return b->finfo[(size_t)file].open_ok ? WVG_OK : WVG_ERR_OPEN;
}

int wvg_batch_file_infos(const wvg_batch *b, int first, int n, wvg_file_info *infos) {
    if (!b || !infos || first < 0 || n < 0) return WVG_ERR_ARG;
    const int have = (int)b->infos.size();
    const int m = first >= have ? 0 : (n < have - first ? n : have - first);
    if (m > 0) memcpy(infos, b->infos.data() + first, sizeof(wvg_file_info) * (size_t)m);
    return m;
}

int wvg_batch_lane_groups(const wvg_batch *b, uint32_t *mask) {
    if (!b || !mask) return WVG_ERR_ARG;
    *mask = b->lane_groups;
    return WVG_OK;
}

int wvg_batch_framing_stats(const wvg_batch *b, int64_t *device_files, int64_t *host_files) {
    if (!b) return WVG_ERR_ARG;
    if (device_files) *device_files = b->framed_dev;
    if (host_files) *host_files = b->framed_host;
    return WVG_OK;
}

// Sort each term-set list (longest blocks first) and build the lane kernels' order of
// it (wvg_batch::ts_lane): called by the upload before it sizes its staging.
static void build_lane_orders(wvg_batch *b) {
    // Each list by length (longest first), then payload bytes per frame.  The lane
    // order (d_ts[t] + n; a lane kernel decodes 64 consecutive entries per wave):
    //  * blocks of under half a payload bit per frame -- digital silence, one zero run
    //    -- in waves of their own (padded with kLaneGap to the next 64), where every
    //    group is one bulk step of the runs (wv_lane.h): a silent block in a wave of
    //    music would hold that wave to the run-aware words for the whole block;
    //  * the others in list order, so that blocks of one kind share waves: full-scale
    //    noise (large medians: the split words) with noise, music with music -- a wave's
    //    time is its slowest lane's.
    auto by_len_density = [&](uint32_t x, uint32_t y) {
        const BlockDesc &p = b->fo.descs[x], &q = b->fo.descs[y];
        if (p.nframes != q.nframes) return p.nframes > q.nframes;
        const uint64_t dp = (uint64_t)p.bits_len * q.nframes, dq = (uint64_t)q.bits_len * p.nframes;
        return dp != dq ? dp < dq : x < y;
    };
    auto silent = [&](uint32_t k) { return (uint64_t)b->fo.descs[k].bits_len * 16u < b->fo.descs[k].nframes; };
    auto pad = [](std::vector<uint32_t> &v) {
        while (v.size() & 63u) v.push_back(kLaneGap);
    };
    // The run-time list kernel's groups (lane_rt_group) are ordered by list first --
    // mono / stereo, lossless / hybrid, length, terms -- each list in waves of its own: a
    // wave decodes the list (and kind) of its first block and hands back any other.
    auto lkey = [&](uint32_t k) {
        const BlockDesc &d = b->fo.descs[k];
        std::array<int8_t, MAXP + 2> key{};
        key[0] = (int8_t)(((d.flags & wvf::MONO_DATA) ? 1 : 0) | ((d.flags & wvf::HYBRID_FLAG) ? 2 : 0));
        key[1] = (int8_t)d.num_terms;
        for (int i = 0; i < d.num_terms && i < MAXP; i++) key[2 + i] = d.term[i];
        return key;
    };
    std::vector<uint32_t> rest, part;
    for (int t = 0; t < kMaxTermSets; t++) {
        std::vector<uint32_t> &L = b->ts_list[t], &LL = b->ts_lane[t];
        LL.clear();
        if (L.empty()) continue;
        std::sort(L.begin(), L.end(), by_len_density);
        // (the keys once per block, then a stable sort of positions by key: the list order --
        // longest first -- stays within each list)
        const bool rt = lane_rt_group(t);
        std::vector<std::array<int8_t, MAXP + 2>> keys;
        std::vector<uint32_t> order = L;
        if (rt) {
            keys.reserve(L.size());
            for (uint32_t k : L) keys.push_back(lkey(k));
            std::vector<uint32_t> pos(L.size());
            for (size_t i = 0; i < pos.size(); i++) pos[i] = (uint32_t)i;
            std::stable_sort(pos.begin(), pos.end(), [&](uint32_t x, uint32_t y) { return keys[x] < keys[y]; });
            std::vector<std::array<int8_t, MAXP + 2>> sk(pos.size());
            for (size_t i = 0; i < pos.size(); i++) {
                order[i] = L[pos[i]];
                sk[i] = keys[pos[i]];
            }
            keys.swap(sk);
        }
        for (size_t i = 0; i < order.size();) {
            size_t j = i + 1;
            if (rt)
                while (j < order.size() && keys[j] == keys[i]) j++;
            else
                j = order.size();
            part.clear();
            rest.clear();
            for (size_t k = i; k < j; k++) (silent(order[k]) ? part : rest).push_back(order[k]);
            if (!part.empty() && !rest.empty()) pad(part);
            part.insert(part.end(), rest.begin(), rest.end());
            if (!LL.empty()) pad(LL);
            LL.insert(LL.end(), part.begin(), part.end());
            i = j;
        }
        while (!LL.empty() && LL.back() == kLaneGap) LL.pop_back();
    }
}

int wvg_batch_upload(wvg_batch *b) {
    if (!b) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    hipStream_t s = b->stream;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, quiesce(b));  // earlier work on these buffers, on the batch's or a caller's stream
    static const bool trace = getenv("WVG_DFRAME_TRACE") && getenv("WVG_DFRAME_TRACE")[0] == '1';
    const double t_up0 = now_ms();
    b->formatted = false;
    // the blob is followed by 64 B of 0xFF (the reader's past-end fill)
    HIPCHK(c, blob_push(b));  // what the adds have not sent yet
    if (!b->d_blob) HIPCHK(c, ensure(b->d_blob, b->cap_blob, 64));
    HIPCHK(c, hipMemsetAsync(b->d_blob + b->blob.size(), 0xFF, 64, s));
    if (!b->dfiles.empty()) {
        const int rc = device_frame(b, s);
        if (rc != WVG_OK) return rc;
    }
    const size_t nd = b->fo.descs.size();
    // The small host arrays go through one page-locked staging buffer: a
    // pageable hipMemcpyAsync is staged synchronously inside the runtime, which
    // serialises host threads serving other batches.  Sized up front (a grow
    // would move the source of copies already queued); the synchronize above
    // means no earlier copy still reads it.
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t need = al(sizeof(BlockDesc) * nd) + al(sizeof(MetaItem) * b->fo.items.size()) +
                  al(sizeof(MetaJob) * b->fo.jobs.size()) + al(b->fo.tables.size()) + al(sizeof(uint32_t) * (nd + 1)) +
                  al(sizeof(uint32_t) * b->pcm_list.size()) + al(sizeof(uint32_t) * b->dsd_list.size()) +
                  al(sizeof(ZeroSeg) * b->fo.zeros.size()) + al(sizeof(FormatSeg) * b->segs.size());
    build_lane_orders(b);
    for (int t = 0; t < kMaxTermSets; t++)
        need += al(sizeof(uint32_t) * b->ts_list[t].size()) + al(sizeof(uint32_t) * b->ts_lane[t].size());
    if (!b->stage.resize(need)) return WVG_ERR_SPACE;
    size_t soff = 0;
    auto put = [&](void *dst, const void *src, size_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        if (soff + bytes > need) {  // (cannot happen: `need` covers every put; never write past the stage)
            soff = need + 1;
            return hipErrorInvalidValue;
        }
        uint8_t *h = b->stage.data() + soff;
        memcpy(h, src, bytes);
        soff += al(bytes);
        return hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s);
    };
    HIPCHK(c, ensure(b->d_descs, b->cap_descs, sizeof(BlockDesc) * (nd ? nd : 1)));
    {   // the host-framed descriptors, around the device-framed runs, which are copied on the device
        size_t k = 0;
        for (const auto &r : b->dev_runs) {
            HIPCHK(c, put(b->d_descs + k, b->fo.descs.data() + k, sizeof(BlockDesc) * (r.dst - k)));
            HIPCHK(c, hipMemcpyAsync(b->d_descs + r.dst, b->d_ddescs + r.src, sizeof(BlockDesc) * r.n,
                                     hipMemcpyDeviceToDevice, s));
            k = r.dst + r.n;
        }
        HIPCHK(c, put(b->d_descs + k, b->fo.descs.data() + k, sizeof(BlockDesc) * (nd - k)));
    }
    if (!b->fo.jobs.empty()) {  // device-side metadata parse: finishes the descriptors in place
        const size_t ni = b->fo.items.size(), nj = b->fo.jobs.size();
        HIPCHK(c, ensure(b->d_items, b->cap_items, sizeof(MetaItem) * ni));
        HIPCHK(c, ensure(b->d_jobs, b->cap_jobs, sizeof(MetaJob) * nj));
        HIPCHK(c, put(b->d_items, b->fo.items.data(), sizeof(MetaItem) * ni));
        HIPCHK(c, put(b->d_jobs, b->fo.jobs.data(), sizeof(MetaJob) * nj));
        HIPCHK(c, launch_meta(b->d_descs, b->d_jobs, (uint32_t)nj, b->d_items, b->d_blob, s));
    }
    HIPCHK(c, ensure(b->d_tables, b->cap_tables, b->fo.tables.size() + 16));
    HIPCHK(c, put(b->d_tables, b->fo.tables.data(), b->fo.tables.size()));
    const size_t no = (size_t)(b->out_ints ? b->out_ints : 1);
    HIPCHK(c, ensure(b->d_out, b->cap_out, sizeof(int32_t) * no));
    HIPCHK(c, hipMemsetAsync(b->d_out, 0, sizeof(int32_t) * no, s));
    size_t cst = b->cap_st;
    HIPCHK(c, ensure(b->d_status, cst, sizeof(uint32_t) * (nd ? nd : 1)));
    HIPCHK(c, ensure(b->d_mute, b->cap_st, sizeof(uint32_t) * (nd ? nd : 1)));
    b->h_status.assign(nd ? nd : 1, 0);
    for (size_t k = 0; k < nd; k++) b->h_status[k] = b->fo.descs[k].fstatus;
    HIPCHK(c, put(b->d_status, b->h_status.data(), sizeof(uint32_t) * b->h_status.size()));
    HIPCHK(c, hipMemsetAsync(b->d_mute, 0, sizeof(uint32_t) * (nd ? nd : 1), s));
    // longest blocks first within a kind, so the long tail starts early (order is
    // free: every block writes its own output range; DSD fills follow on the same stream)
    // (KIND_SKIP first: the mode-3 range [dsd_high_lo, end) then holds mode-3 blocks only)
    auto kind_rank = [](uint32_t k) { return k == KIND_SKIP ? 0u : k + 1u; };
    auto by_kind_len = [&](uint32_t x, uint32_t y) {
        const BlockDesc &p = b->fo.descs[x], &q = b->fo.descs[y];
        if (p.kind != q.kind) return kind_rank(p.kind) < kind_rank(q.kind);
        if (p.kind == KIND_DSD_HIGH || p.kind == KIND_DSD_FAST) {  // stereo before mono (one lane kernel each)
            const bool pm = (p.flags & wvf::MONO_DATA) != 0, qm = (q.flags & wvf::MONO_DATA) != 0;
            if (pm != qm) return qm;
        }
        return p.nframes != q.nframes ? p.nframes > q.nframes : x < y;
    };
    std::sort(b->pcm_list.begin(), b->pcm_list.end(), by_kind_len);
    // the .wvc lane kernel's candidates at the tail (longest first there too)
    b->pcm_wvc_n = (uint32_t)(b->pcm_list.end() -
                              std::stable_partition(b->pcm_list.begin(), b->pcm_list.end(), [&](uint32_t k) {
                                  return !wvc_lane_candidate(b->fo.descs[k]);
                              }));
    std::sort(b->dsd_list.begin(), b->dsd_list.end(), by_kind_len);
    // the mode-1 blocks are one range of the kind-sorted list (their own kernel)
    b->dsd_fast_lo = b->dsd_fast_n = b->dsd_fast_mono = 0;
    b->dsd_high_lo = (uint32_t)b->dsd_list.size();
    b->dsd_high_mono = 0;
    for (size_t k = 0; k < b->dsd_list.size(); k++) {
        const BlockDesc &d = b->fo.descs[b->dsd_list[k]];
        if (d.kind == KIND_DSD_HIGH) {
            if (b->dsd_high_lo == b->dsd_list.size()) b->dsd_high_lo = (uint32_t)k;
            if (d.flags & wvf::MONO_DATA) b->dsd_high_mono++;
        }
        if (d.kind != KIND_DSD_FAST) continue;
        if (!b->dsd_fast_n) b->dsd_fast_lo = (uint32_t)k;
        b->dsd_fast_n++;
        if (d.flags & wvf::MONO_DATA) b->dsd_fast_mono++;
    }
    const size_t np = b->pcm_list.size(), ns = b->dsd_list.size();
    HIPCHK(c, ensure(b->d_pcml, b->cap_pcml, sizeof(uint32_t) * (np ? np : 1)));
    HIPCHK(c, ensure(b->d_dsd, b->cap_dsd, sizeof(uint32_t) * (ns ? ns : 1)));
    HIPCHK(c, put(b->d_pcml, b->pcm_list.data(), sizeof(uint32_t) * np));
    b->nzeros = (uint32_t)b->fo.zeros.size();
    if (b->nzeros) {
        HIPCHK(c, ensure(b->d_zeros, b->cap_zeros, sizeof(ZeroSeg) * b->nzeros));
        HIPCHK(c, put(b->d_zeros, b->fo.zeros.data(), sizeof(ZeroSeg) * b->nzeros));
    }
    HIPCHK(c, put(b->d_dsd, b->dsd_list.data(), sizeof(uint32_t) * ns));
    for (int t = 0; t < kMaxTermSets; t++) {
        const std::vector<uint32_t> &L = b->ts_list[t], &LL = b->ts_lane[t];
        if (L.empty()) continue;
        HIPCHK(c, ensure(b->d_ts[t], b->cap_ts[t], sizeof(uint32_t) * (L.size() + LL.size())));
        HIPCHK(c, put(b->d_ts[t], L.data(), sizeof(uint32_t) * L.size()));
        HIPCHK(c, put(b->d_ts[t] + L.size(), LL.data(), sizeof(uint32_t) * LL.size()));
    }
    // the WavpackFormatSamples segments (wvg_batch_format), so a format issues no copy of its own
    HIPCHK(c, ensure(b->d_segs, b->cap_segs, sizeof(FormatSeg) * (b->segs.empty() ? 1 : b->segs.size())));
    HIPCHK(c, put(b->d_segs, b->segs.data(), sizeof(FormatSeg) * b->segs.size()));
    if (soff > need) {  // (cannot happen: the sizes above cover every put)
        c->err = "upload: staging buffer undersized";
        return WVG_ERR_HIP;
    }
    // frames per launch group: the load the decode's lane assignment balances
    auto frames_of = [&](const std::vector<uint32_t> &L) {
        int64_t f = 0;
        for (uint32_t k : L) f += b->fo.descs[k].nframes;
        return f;
    };
    for (int t = 0; t < kMaxTermSets; t++) b->gframes[t] = frames_of(b->ts_list[t]);
    b->gframes[kMaxTermSets] = frames_of(b->pcm_list);
    HIPCHK(c, hipEventRecord(b->up, s));  // (a decode on a caller's stream waits for it)
    // No wait for the copies: their sources are the page-locked blob and staging
    // buffers, which change only after a quiesce (reset, the next upload) or, for a
    // blob that must grow, after the copies finished (blob_resize).  The caller's
    // thread goes on to its next request while this one's DMA runs.
    if (trace) {
        HIPCHK(c, hipStreamSynchronize(s));
        fprintf(stderr, "upload: %.3f ms (%zu blocks)\n", now_ms() - t_up0, nd);
    }
    b->uploaded = true;
    b->downloaded = false;
    b->segs_uploaded = false;
    return WVG_OK;
}

static hipError_t take_event(wvg_batch *b, hipEvent_t *e) {
    if (!b->tfree.empty()) {
        *e = b->tfree.back();
        b->tfree.pop_back();
        return hipSuccess;
    }
    return hipEventCreate(e);
}

// Fold the oldest `pairs` pending timing pairs into t_sum/t_cnt (waits for them).
static hipError_t fold_timing(wvg_batch *b, int pairs) {
    for (int i = 0; i < pairs; i++) {
        float t = 0;
        hipError_t e = hipEventSynchronize(b->tev[2 * i + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&t, b->tev[2 * i], b->tev[2 * i + 1]);
        if (e != hipSuccess) return e;
        b->t_sum += t;
        b->t_cnt++;
        b->tfree.push_back(b->tev[2 * i]);
        b->tfree.push_back(b->tev[2 * i + 1]);
    }
    b->tev.erase(b->tev.begin(), b->tev.begin() + 2 * pairs);
    return hipSuccess;
}

// the other batches of b's context with a decode or format still running
static int others_running(wvg_batch *b) {
    std::lock_guard<std::mutex> g(b->ctx->mu);
    int k = 0;
    for (wvg_batch *o : b->ctx->batches)
        if (o != b && o->done && hipEventQuery(o->done) == hipErrorNotReady) k++;
    return k;
}

int wvg_batch_decode(wvg_batch *b, void *stream) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));  // side streams and events belong to the batch's device, whatever the calling thread
    hipStream_t s = stream ? (hipStream_t)stream : b->stream;
    if (s != b->stream) HIPCHK(c, hipStreamWaitEvent(s, b->up, 0));  // the upload's copies (not waited for)
    if (b->timing) {
        // a bounded number of pairs stays pending: the oldest is folded into the
        // running sum (it finished long ago) and its events are reused
        if (b->tev.size() >= 2 * kTimingPending) HIPCHK(c, fold_timing(b, 1));
        hipEvent_t e0, e1;
        HIPCHK(c, take_event(b, &e0));
        HIPCHK(c, take_event(b, &e1));
        b->tev.push_back(e0);
        b->tev.push_back(e1);
        HIPCHK(c, hipEventRecord(e0, s));
    }
    // The non-empty launch groups (DSD, DSD mode 1, generic PCM, term sets 0..7)
    // each go onto a stream of their own when the decode is issued alone (its
    // batch's stream and the context's side streams).  Streams beyond the process's
    // hardware queues (GPU_MAX_HW_QUEUES, the host's choice) share a queue, whose
    // kernels then run one after another -- a PCM group queued behind the DSD group
    // (its mode-3 blocks are the batch's longest serial chains) waits for all of it.
    // With fewer lanes than groups the DSD groups keep lanes of their own and the
    // PCM groups share the rest, the largest first onto the least loaded.
    const int kDsd = kMaxTermSets + 1, kDsd1 = kMaxTermSets + 2, kPcm = kMaxTermSets;
    int used[kSide], n = 0;
    if (!b->dsd_list.empty() && b->dsd_fast_n < b->dsd_list.size()) used[n++] = kDsd;
    if (b->dsd_fast_n) used[n++] = kDsd1;
    if (!b->pcm_list.empty()) used[n++] = kPcm;
    for (int t = 0; t < kMaxTermSets; t++)
        if (!b->ts_list[t].empty()) used[n++] = t;
    int lane_of[kSide];
    // With other batches of this context running, a decode's groups share the
    // hardware queues with theirs: it takes streams of its own (its stream and up to
    // kLanes - 1 side streams of the batch) only as far as the queue budget leaves
    // each batch in flight, else everything goes in order onto its one stream (the
    // batches in flight fill the device).  One stream per batch: C5's 4,000-file
    // slice at 20 in flight 10,600 Mframes/s against 6,500 on one stream per group
    // (profiles/r04_c5_streams.txt); 25 slices on 24 queues with a second stream
    // each for the DSD groups: 7,446 -> 9,337 Msamples/s, but the 4,000-file slice at
    // 20 in flight 13,174 -> 11,148 (40 streams on 24 queues,
    // profiles/r05_c5_streams.jsonl) -- hence the budget.
    // (asked when it decides something: a multi-group decode's streams, or the default
    // kernel choice -- also while the hold is on, so that batches that keep overlapping
    // keep renewing it: the hold is a sliding window over the last overlap seen)
    const double t_now = now_ms();
    const bool held = t_now - c->concurrent_ms.load() < kConcurrentHoldMs;
    const bool ask = (!b->lanes_env && b->lanes > 1 && n > 1) || b->kernel_auto;
    const int others = ask ? others_running(b) : 0;
    const bool running = others > 0;
    int nlanes = b->lanes;
    bool has_pcm = !b->pcm_list.empty();
    for (int t = 0; t < kMaxTermSets; t++) has_pcm |= !b->ts_list[t].empty();
    int own = 1;  // streams of its own while others run
    if (running && !b->lanes_env && n > 1) {
        if (c->own_streams < 0) {
            own = c->hw_queues / (others + 1);
            own = own < 1 ? 1 : (own > kLanes ? kLanes : own);
        } else if (c->own_streams == 1 && !b->dsd_list.empty() && has_pcm) {
            own = 2;  // (WVG_DSD_STREAM=1: the DSD groups on a second stream whatever the budget)
        }
    }
    const bool own_side = running && own > 1;
    if (!b->lanes_env && nlanes > 1 && running) nlanes = own;
    // WVG_KERNEL_AUTO: in a context that has had batches in flight together, the lane
    // kernels (throughput) -- for kConcurrentHoldMs after a decode last found another
    // batch running; in one that decodes a batch at a time, a group of at most
    // kAutoLaneMin blocks on the one-workgroup / one-wave-per-block kernels, whose chains
    // run faster than a lane's (C2 alone: 6.5 vs 7.5 ms; C4 15.4 vs 24.4; DSD mode 3 34 vs
    // 56), larger ones on lanes (C3's 4,096 blocks: 24.8 vs 37.7 ms).  (Not per decode: a
    // lane workgroup needs a whole CU's LDS, and a two-wave decode among lane decodes
    // leaves CUs partly taken -- C4 at 20 in flight fell from 16,000 to 8,200 Mframes/s
    // when the first decode of each round ran alone on the two-wave kernel.)
    if (running) c->concurrent_ms = t_now;
    const bool lanes_now = running || held;
    auto mode_of = [&](size_t nblocks) -> int {
        if (!b->kernel_auto) return b->lane_mode;
        return (lanes_now || nblocks > kAutoLaneMin) ? 1 : 0;
    };
    // (WVG_DSD3_WAVE=1: DSD mode 3 on the wave-per-block kernel whatever the PCM groups use -- A/B)
    static const bool dsd3_wave = getenv("WVG_DSD3_WAVE") && getenv("WVG_DSD3_WAVE")[0] == '1';
    const int dsd3_mode = dsd3_wave ? 0 : mode_of(b->dsd_list.size() - b->dsd_high_lo);
    if (b->log_decodes)
        fprintf(stderr, "wvg decode %p: groups %d, others running %d, streams %d, own %d, auto %d\n", (void *)b, n,
                others, nlanes < n ? nlanes : n, (int)own_side, (int)b->kernel_auto);
    const int nl = n < nlanes ? n : nlanes;
    if (n <= nlanes) {
        for (int i = 0; i < n; i++) lane_of[used[i]] = i;
    } else {
        int64_t load[kSide] = {0};
        int first = 0;  // lanes before it are reserved for the DSD groups
        // (DSD mode 3 first -- the batch's longest chains -- then mode 1, each while a lane
        // is left for the rest; a DSD group without a lane of its own joins the PCM
        // groups' pool, placed first; with a single lane everything is on it)
        bool pooled[kSide] = {false};
        for (int g : {kDsd, kDsd1})
            for (int i = 0; i < n; i++)
                if (used[i] == g) {
                    if (first < nl - 1) lane_of[g] = first++;
                    else pooled[g] = true;
                }
        int pcm[kSide], np = 0;
        for (int i = 0; i < n; i++)
            if ((used[i] != kDsd && used[i] != kDsd1) || pooled[used[i]]) pcm[np++] = used[i];
        auto load_of = [&](int g) -> int64_t { return (g == kDsd || g == kDsd1) ? INT64_MAX / 4 : b->gframes[g]; };
        std::sort(pcm, pcm + np, [&](int x, int y) { return load_of(x) > load_of(y); });
        for (int i = 0; i < np; i++) {
            int best = first;
            for (int l = first; l < nl; l++)
                if (load[l] < load[best]) best = l;
            lane_of[pcm[i]] = best;
            load[best] += load_of(pcm[i]);
        }
    }
    hipStream_t side[kLanes - 1] = {nullptr};
    for (int l = 1; l < nl; l++) {
        if (own_side) {  // (the batch's own side streams, not the context's shared ones)
            if (!b->dstream[l - 1]) HIPCHK(c, hipStreamCreateWithFlags(&b->dstream[l - 1], hipStreamNonBlocking));
            side[l - 1] = b->dstream[l - 1];
        } else {
            std::lock_guard<std::mutex> g(c->mu);
            if (!c->side[l - 1]) HIPCHK(c, hipStreamCreateWithFlags(&c->side[l - 1], hipStreamNonBlocking));
            side[l - 1] = c->side[l - 1];
        }
        if (!b->join[l - 1]) HIPCHK(c, hipEventCreateWithFlags(&b->join[l - 1], hipEventDisableTiming));
    }
    auto lane = [&](int l) -> hipStream_t { return l == 0 ? s : side[l - 1]; };
    auto slot = [&](int g) -> hipStream_t {
        for (int i = 0; i < n; i++)
            if (used[i] == g) return lane(lane_of[g]);
        return s;  // (an empty group launches nothing)
    };
    // the gap zero-fills (WavPackUtils.cs:227-251) are part of the decode's output
    if (b->nzeros) HIPCHK(c, launch_zero_fill(b->d_zeros, b->nzeros, b->d_out, s));
    if (nl > 1) {
        HIPCHK(c, hipEventRecord(b->fork, s));
        for (int l = 1; l < nl; l++) HIPCHK(c, hipStreamWaitEvent(lane(l), b->fork, 0));
    }
    if (b->timing) {
        b->gstart = b->tev[b->tev.size() - 2];
        b->gmask = 0;
    }
    // per-group end times (timing on): an event on the group's lane right after its launch
    auto mark = [&](int g) -> hipError_t {
        if (!b->timing) return hipSuccess;
        for (int i = 0; i < n; i++) {
            if (used[i] != g) continue;
            if (!b->gev[g]) {
                hipError_t e = hipEventCreate(&b->gev[g]);
                if (e != hipSuccess) return e;
            }
            b->gmask |= 1u << g;
            return hipEventRecord(b->gev[g], slot(g));
        }
        return hipSuccess;
    };
    HIPCHK(c, launch_decode(b->d_descs, b->d_pcml, (uint32_t)b->pcm_list.size(), b->d_dsd, (uint32_t)b->dsd_list.size(),
                            b->dsd_fast_lo, b->dsd_fast_n, b->d_blob, b->d_tables, b->d_out, b->d_status, b->d_mute,
                            slot(kPcm), slot(kDsd), slot(kDsd1), dsd3_mode,
                            b->dsd_high_lo, b->dsd_high_mono, mode_of(b->dsd_fast_n), b->dsd_fast_mono,
                            // (.wvc blocks: the lane kernel even alone -- 35.8 against the generic
                            // kernel's 130 ms for C4's 1,024 blocks, profiles/r05_c4wvc_rates.jsonl)
                            b->kernel_auto ? 1 : b->lane_mode, b->pcm_wvc_n));
    {   // the launch groups this decode gave to lane / row kernels (wvg_batch_lane_groups)
        uint32_t m = 0;
        for (int t = 0; t < kMaxTermSets; t++)
            if (!b->ts_list[t].empty() && mode_of(b->ts_list[t].size())) m |= 1u << t;
        if (b->pcm_wvc_n && (b->kernel_auto || b->lane_mode)) m |= 1u << kPcm;
        if (b->dsd_list.size() > b->dsd_high_lo && dsd3_mode) m |= 1u << kDsd;
        if (b->dsd_fast_n && mode_of(b->dsd_fast_n)) m |= 1u << kDsd1;
        b->lane_groups = m;
    }
    HIPCHK(c, mark(kDsd));
    HIPCHK(c, mark(kDsd1));
    HIPCHK(c, mark(kPcm));
    for (int t = 0; t < kMaxTermSets; t++)
        if (!b->ts_list[t].empty()) {
            HIPCHK(c, launch_2wave(t, b->d_descs, b->d_ts[t], (uint32_t)b->ts_list[t].size(), b->d_blob, b->d_out,
                                   b->d_status, b->d_mute, slot(t), mode_of(b->ts_list[t].size()),
                                   b->d_ts[t] + b->ts_list[t].size(),
                                   (uint32_t)b->ts_lane[t].size(),
                                   b->d_lane_dbg && b->ts_lane[t].size() <= 64u * kLaneDbgWaves
                                       ? b->d_lane_dbg + (size_t)t * kLaneDbgWaves * 16u
                                       : nullptr));
            HIPCHK(c, mark(t));
        }
    for (int l = 1; l < nl; l++) {
        HIPCHK(c, hipEventRecord(b->join[l - 1], lane(l)));
        HIPCHK(c, hipStreamWaitEvent(s, b->join[l - 1], 0));
    }
    HIPCHK(c, launch_dsd_fill(b->d_descs, b->d_dsd, (uint32_t)b->dsd_list.size(), b->d_status, b->d_mute, b->d_out, s));
    if (b->timing) HIPCHK(c, hipEventRecord(b->tev.back(), s));
    HIPCHK(c, hipEventRecord(b->done, s));
    b->downloaded = false;
    b->formatted = false;
    return WVG_OK;
}

int wvg_batch_sync(wvg_batch *b) {
    if (!b) return WVG_ERR_ARG;
    HIPCHK(b->ctx, hipEventSynchronize(b->done));
    HIPCHK(b->ctx, hipStreamSynchronize(b->stream));
    return WVG_OK;
}

void *wvg_batch_stream(wvg_batch *b) { return b ? (void *)b->stream : nullptr; }

int wvg_batch_poison(wvg_batch *b, int byte) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, quiesce(b));
    if (b->out_ints) HIPCHK(c, hipMemsetAsync(b->d_out, byte & 0xFF, sizeof(int32_t) * (size_t)b->out_ints, b->stream));
    const size_t nd = b->fo.descs.size();
    if (nd) {
        // every block a kernel decodes gets WVG_ST_UNWRITTEN until a decode stores its status
        // (KIND_SKIP blocks keep the framing's verdict: no kernel writes them)
        std::vector<uint32_t> st(nd);
        for (size_t k = 0; k < nd; k++)
            st[k] = b->fo.descs[k].fstatus | (b->fo.descs[k].kind == KIND_SKIP ? 0u : (uint32_t)WVG_ST_UNWRITTEN);
        HIPCHK(c, hipMemcpyAsync(b->d_status, st.data(), sizeof(uint32_t) * nd, hipMemcpyHostToDevice, b->stream));
        HIPCHK(c, hipMemsetAsync(b->d_mute, 0, sizeof(uint32_t) * nd, b->stream));
    }
    HIPCHK(c, hipStreamSynchronize(b->stream));
    b->downloaded = false;
    return WVG_OK;
}

int wvg_batch_set_kernel(wvg_batch *b, int kernel) {
    if (!b || (kernel != WVG_KERNEL_TWO_WAVE && kernel != WVG_KERNEL_LANE && kernel != WVG_KERNEL_AUTO))
        return WVG_ERR_ARG;
    if (kernel == WVG_KERNEL_AUTO) {
        b->kernel_auto = true;
        return WVG_OK;
    }
    b->kernel_auto = false;
    b->lane_mode = kernel == WVG_KERNEL_LANE ? 1 : 0;
    return WVG_OK;
}

int wvg_batch_set_timing(wvg_batch *b, int on) {
    if (!b) return WVG_ERR_ARG;
    // pending pairs are dropped; their events are reused (re-recording an event is allowed)
    b->tfree.insert(b->tfree.end(), b->tev.begin(), b->tev.end());
    b->tev.clear();
    b->t_sum = 0;
    b->t_cnt = 0;
    b->timing = on != 0;
    return WVG_OK;
}

int wvg_batch_timed(wvg_batch *b, float *avg_ms, int *count) {
    if (!b || !avg_ms || !count) return WVG_ERR_ARG;
    HIPCHK(b->ctx, fold_timing(b, (int)(b->tev.size() / 2)));
    *avg_ms = b->t_cnt ? (float)(b->t_sum / b->t_cnt) : 0.f;
    *count = b->t_cnt;
    return WVG_OK;
}

int wvg_batch_group_times(wvg_batch *b, float *ms, int cap) {
    if (!b || !ms || cap < kSide) return WVG_ERR_ARG;
    for (int g = 0; g < kSide; g++) {
        ms[g] = -1.f;
        if (!(b->gmask & (1u << g)) || !b->gstart) continue;
        HIPCHK(b->ctx, hipEventSynchronize(b->gev[g]));
        HIPCHK(b->ctx, hipEventElapsedTime(&ms[g], b->gstart, b->gev[g]));
    }
    return kSide;
}

int64_t wvg_batch_out_ints(const wvg_batch *b) { return b ? b->out_ints : 0; }
int32_t *wvg_batch_device_out(wvg_batch *b) { return b ? b->d_out : nullptr; }
int64_t wvg_batch_num_blocks(const wvg_batch *b) { return b ? (int64_t)b->fo.descs.size() : 0; }
int64_t wvg_batch_bytes_in(const wvg_batch *b) { return b ? b->bytes_in : 0; }
int64_t wvg_batch_frames(const wvg_batch *b) { return b ? b->frames : 0; }

static int download_status(wvg_batch *b) {
    wvg_ctx *c = b->ctx;
    size_t nd = b->fo.descs.size();
    b->h_status.assign(nd, 0);
    b->h_aux.assign(nd, 0);
    if (nd) {  // through page-locked memory (a pageable copy blocks other host threads' HIP calls)
        if (!b->hst.resize(2 * sizeof(uint32_t) * nd)) return WVG_ERR_SPACE;
        uint32_t *h = (uint32_t *)b->hst.data();
        HIPCHK(c, hipStreamWaitEvent(b->stream, b->done, 0));
        HIPCHK(c, hipMemcpyAsync(h, b->d_status, sizeof(uint32_t) * nd, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(c, hipMemcpyAsync(h + nd, b->d_mute, sizeof(uint32_t) * nd, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(c, hipStreamSynchronize(b->stream));
        memcpy(b->h_status.data(), h, sizeof(uint32_t) * nd);
        memcpy(b->h_aux.data(), h + nd, sizeof(uint32_t) * nd);
    }
    b->downloaded = true;
    return WVG_OK;
}

int wvg_batch_download(wvg_batch *b, int32_t *host_out, int64_t cap_ints) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamWaitEvent(b->stream, b->done, 0));  // the decode, on whatever stream it ran
    if (!host_out && cap_ints == -1) {  // into the batch's page-locked buffer (wvg_batch_host_out)
        if (!b->hout.resize(sizeof(int32_t) * (size_t)(b->out_ints ? b->out_ints : 1))) return WVG_ERR_SPACE;
        host_out = (int32_t *)b->hout.data();
        cap_ints = b->out_ints;
    }
    if (host_out) {
        if (cap_ints < b->out_ints) return WVG_ERR_SPACE;
        if (b->out_ints)
            HIPCHK(c, hipMemcpyAsync(host_out, b->d_out, sizeof(int32_t) * (size_t)b->out_ints, hipMemcpyDeviceToHost,
                                     b->stream));
    }
    return download_status(b);
}

int32_t *wvg_batch_host_out(wvg_batch *b) { return b && !b->hout.empty() ? (int32_t *)b->hout.data() : nullptr; }

int wvg_batch_lane_counters(wvg_batch *b, int ts, uint32_t *out, int64_t cap) {
    if (!b || ts < 0 || ts >= kMaxTermSets || !b->d_lane_dbg) return WVG_ERR_ARG;
    const size_t nw = (b->ts_lane[ts].size() + 63) / 64;
    if (nw > kLaneDbgWaves) return WVG_ERR_ARG;
    if (cap < (int64_t)(16 * nw)) return WVG_ERR_SPACE;
    // (the decode may have run on a caller's stream or the context's side streams)
    HIPCHK(b->ctx, hipEventSynchronize(b->done));
    HIPCHK(b->ctx, hipStreamSynchronize(b->stream));
    HIPCHK(b->ctx, hipMemcpy(out, b->d_lane_dbg + (size_t)ts * kLaneDbgWaves * 16u, sizeof(uint32_t) * 16 * nw,
                             hipMemcpyDeviceToHost));
    return (int)nw;
}

int wvg_batch_block_status(wvg_batch *b, uint32_t *out, int64_t cap) {
    if (!b || !b->downloaded) return WVG_ERR_ARG;
    int64_t n = (int64_t)b->h_status.size();
    if (cap < n) return WVG_ERR_SPACE;
    if (n) memcpy(out, b->h_status.data(), sizeof(uint32_t) * (size_t)n);
    return (int)n;
}

// the file's first block that raised the reference's exception (-1: none)
static int64_t first_exception_block(const wvg_batch *b, const FileInfo &fi) {
    for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++)
        if (b->h_status[(size_t)k] & ST_EXCEPTION) return k;
    return -1;
}

// frames the file's calls return before the call that throws: the call holding the
// device-reported frame of the first block that raised (-1: no device exception)
static int64_t exception_call_frame(const wvg_batch *b, const FileInfo &fi, const wvg_file_info &wi) {
    const int64_t kx = first_exception_block(b, fi);
    if (kx < 0) return -1;
    const int nch = wi.reduced_channels ? wi.reduced_channels : 1;
    const BlockDesc &d = b->fo.descs[(size_t)kx];
    const int64_t start = ((int64_t)d.out_off - wi.out_offset) / nch;  // block's first output frame
    const int64_t t = b->h_aux[(size_t)kx];
    if (t < (int64_t)d.first_chunk) return start - (int64_t)d.first_bsp / nch;
    return start + d.first_chunk + (t - d.first_chunk) / d.chunk * d.chunk;
}

// the status word a block contributes to the file result
static uint32_t block_verdict(const wvg_batch *b, int64_t k) {
    const BlockDesc &d = b->fo.descs[(size_t)k];
    // (which kernel decoded it is not a result, nor is the poison bit of wvg_batch_poison)
    uint32_t st = b->h_status[(size_t)k] & ~((uint32_t)ST_REDONE | (uint32_t)WVG_ST_UNWRITTEN);
    // a block decoded from state the device cannot see (only in malformed
    // files): the reference decodes garbage and its CRC check fails
    if ((st & ST_UNSUPPORTED) && d.nframes == d.block_samples) st |= ST_CRC_CHECKED | ST_CRC_ERROR;
    return st;
}

int wvg_batch_file_result(wvg_batch *b, int file, wvg_file_result *res) {
    if (!b || !b->downloaded || file < 0 || file >= (int)b->finfo.size() || !res) return WVG_ERR_ARG;
    const FileInfo &fi = b->finfo[(size_t)file];
    memset(res, 0, sizeof(*res));
    res->frames = fi.out_frames;
    res->exception = fi.exception;
    res->exception_frame = -1;
    res->num_blocks = (int32_t)fi.num_desc;
    res->lossy = fi.lossy_blocks || (fi.config_flags & 8) != 0;
    bool timeout = false;
    for (int64_t k = fi.first_desc; k < fi.first_desc + fi.num_desc; k++) {
        const uint32_t st = block_verdict(b, k);
        res->status_or |= st;
        if (st & ST_TIMEOUT) timeout = true;
        if (st & ST_CRC_ERROR) res->crc_errors++;
        if (st & ST_EXCEPTION) {
            res->exception = 1;
            break;
        }
    }
    if (res->exception) {
        res->exception_frame = exception_call_frame(b, fi, b->infos[(size_t)file]);
        if (res->exception_frame < 0 || res->exception_frame > fi.out_frames) res->exception_frame = fi.out_frames;
        res->frames = -1;
    }
    if (timeout) {
        b->ctx->err = "a decode kernel's bounded wait ran out (ST_TIMEOUT): output of this file is invalid";
        return WVG_ERR_TIMEOUT;
    }
    return WVG_OK;
}

int wvg_batch_file_blocks(wvg_batch *b, int file, int64_t *end_frame, uint32_t *status, int64_t cap) {
    if (!b || !b->downloaded || file < 0 || file >= (int)b->finfo.size()) return WVG_ERR_ARG;
    const FileInfo &fi = b->finfo[(size_t)file];
    const wvg_file_info &wi = b->infos[(size_t)file];
    if (cap < fi.num_desc) return WVG_ERR_SPACE;
    const int nch = wi.reduced_channels ? wi.reduced_channels : 1;
    for (int64_t k = 0; k < fi.num_desc; k++) {
        const BlockDesc &d = b->fo.descs[(size_t)(fi.first_desc + k)];
        // out_off is the block's first output frame (a seek's dropped frames lie before the file's output)
        const int64_t start = ((int64_t)d.out_off - wi.out_offset) / nch;
        if (end_frame) end_frame[k] = start + (int64_t)d.nframes;
        if (status) status[k] = block_verdict(b, fi.first_desc + k);
    }
    return (int)fi.num_desc;
}

int wvg_batch_time(wvg_batch *b, int iters, float *ms) {
    // mean device time of one decode launch: an event pair around each launch on
    // the decode stream, so launch gaps between iterations are not counted
    if (!b || !b->uploaded || iters <= 0) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    std::vector<hipEvent_t> ev((size_t)iters * 2);
    for (auto &e : ev) HIPCHK(c, hipEventCreate(&e));
    for (int i = 0; i < iters; i++) {
        HIPCHK(c, hipEventRecord(ev[2 * i], b->stream));
        int rc = wvg_batch_decode(b, nullptr);
        if (rc) return rc;
        HIPCHK(c, hipEventRecord(ev[2 * i + 1], b->stream));
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

// ---------------------------------------------------------------------------
// WavpackFormatSamples epilogue + the WvDemo .wav image
// ---------------------------------------------------------------------------
int wvg_batch_format(wvg_batch *b, int dsd, void *stream) {
    if (!b || !b->uploaded) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));  // d_pcm is allocated on the batch's device
    hipStream_t s = stream ? (hipStream_t)stream : b->stream;
    if (s != b->stream) HIPCHK(c, hipStreamWaitEvent(s, b->up, 0));  // the segments come with the upload
    HIPCHK(c, hipStreamWaitEvent(s, b->done, 0));
    if (!b->segs_uploaded) {  // once per upload (the segments came with it)
        const size_t pb = (size_t)(b->pcm_bytes ? b->pcm_bytes : 1);
        HIPCHK(c, ensure(b->d_pcm, b->cap_pcm, pb));
        HIPCHK(c, hipMemsetAsync(b->d_pcm, 0, pb, s));
        b->segs_uploaded = true;
    }
    HIPCHK(c, launch_format(b->d_segs, (uint32_t)b->segs.size(), b->d_out, b->d_pcm, dsd ? 1 : 0, s));
    HIPCHK(c, hipEventRecord(b->done, s));
    b->formatted = true;
    return WVG_OK;
}

int64_t wvg_batch_pcm_bytes(const wvg_batch *b) { return b ? b->pcm_bytes : 0; }

int64_t wvg_batch_pcm_offset(const wvg_batch *b, int file) {
    if (!b || file < 0 || file >= (int)b->pcm_off.size()) return WVG_ERR_ARG;
    return b->pcm_off[(size_t)file];
}

uint8_t *wvg_batch_device_pcm(wvg_batch *b) { return b ? b->d_pcm : nullptr; }
uint8_t *wvg_batch_host_pcm(wvg_batch *b) { return b && !b->hpcm.empty() ? b->hpcm.data() : nullptr; }

int wvg_batch_download_pcm(wvg_batch *b, uint8_t *host, int64_t cap) {
    if (!b || !b->formatted) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (!host && cap == -1) {  // into the batch's page-locked buffer (wvg_batch_host_pcm)
        if (!b->hpcm.resize((size_t)(b->pcm_bytes ? b->pcm_bytes : 1))) return WVG_ERR_SPACE;
        host = b->hpcm.data();
        cap = b->pcm_bytes;
    }
    if (!host && b->pcm_bytes) return WVG_ERR_ARG;
    if (cap < b->pcm_bytes) return WVG_ERR_SPACE;
    HIPCHK(c, hipStreamWaitEvent(b->stream, b->done, 0));
    if (b->pcm_bytes)
        HIPCHK(c, hipMemcpyAsync(host, b->d_pcm, (size_t)b->pcm_bytes, hipMemcpyDeviceToHost, b->stream));
    HIPCHK(c, hipStreamSynchronize(b->stream));
    return WVG_OK;
}

int wvg_batch_download_pcm_async(wvg_batch *b) {
    if (!b || !b->formatted) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t nb = (size_t)(b->pcm_bytes ? b->pcm_bytes : 1);
    if (nb > b->hpcm.cap) HIPCHK(c, quiesce(b));  // (a grown buffer is a new one: no DMA may still land in the old)
    if (!b->hpcm.resize(nb)) return WVG_ERR_SPACE;
    HIPCHK(c, hipStreamWaitEvent(b->stream, b->done, 0));
    if (b->pcm_bytes) {
        // (WVG_PCM_DMA=1: the DMA-engine copy instead of the copy kernel -- A/B)
        static const bool dma = getenv("WVG_PCM_DMA") && getenv("WVG_PCM_DMA")[0] == '1';
        void *hdev = nullptr;
        if (!dma && b->hpcm.pinned && hipHostGetDevicePointer(&hdev, b->hpcm.data(), 0) == hipSuccess && hdev)
            HIPCHK(c, launch_copy_to_host(b->d_pcm, (uint8_t *)hdev, (size_t)b->pcm_bytes, b->stream));
        else
            HIPCHK(c, hipMemcpyAsync(b->hpcm.data(), b->d_pcm, (size_t)b->pcm_bytes, hipMemcpyDeviceToHost, b->stream));
    }
    HIPCHK(c, hipEventRecord(b->done, b->stream));  // (wvg_batch_sync and the next quiesce wait for it)
    return WVG_OK;
}

static void put_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// WvDemo.Main (WvDemo.cs:15-168) for file `file` of a formatted batch whose
// chunk is the demo's 4096 (Defines.SAMPLE_BUFFER_SIZE): the bytes it writes
// to the .wav and its exit code.
int wvg_batch_wav(wvg_batch *b, int file, uint8_t *out, int64_t cap, int64_t *wav_len, int32_t *exit_code) {
    if (!b || !b->formatted || file < 0 || file >= (int)b->finfo.size() || !wav_len || !exit_code) return WVG_ERR_ARG;
    wvg_ctx *c = b->ctx;
    const FileInfo &fi = b->finfo[(size_t)file];
    const wvg_file_info &wi = b->infos[(size_t)file];
    *wav_len = 0;
    *exit_code = 1;
    if (!fi.open_ok) return WVG_OK;  // WvDemo.cs:41-46: error message, no .wav
    HIPCHK(c, hipEventSynchronize(b->done));
    if (!b->downloaded) {
        int rc = download_status(b);
        if (rc) return rc;
    }
    wvg_file_result r;
    if (wvg_batch_file_result(b, file, &r) == WVG_ERR_TIMEOUT) return WVG_ERR_TIMEOUT;
    const int nch = wi.reduced_channels, bps = wi.bytes_per_sample;
    const int64_t block_align = (int64_t)bps * nch;
    const int64_t total_native = fi.total_samples * (wi.dsd_multiplier > 0 ? 8 : 1);  // WavpackGetNumSamples(wpc, true)
    const int64_t loop_samples = total_native / 100 / 4096 * 4096;                    // WvDemo.cs:112
    // frames written: whole calls before the one that threw (WvDemo.cs:144 catch)
    int64_t limit = fi.out_frames;
    bool exc = fi.exception != 0;
    const int64_t call = exception_call_frame(b, fi, wi);
    if (call >= 0) {
        limit = call < limit ? call : limit;
        exc = true;
    }
    int64_t frames;
    bool trailer = false;
    int32_t rc = 1;
    if (fi.first_call_frames < 0) {
        frames = 0;  // the first call threw
    } else if (loop_samples == 0) {
        // `total % loop_samples` divides by zero after the first call's write (WvDemo.cs:130)
        frames = limit < fi.first_call_frames ? limit : fi.first_call_frames;
    } else {
        frames = limit;
        if (!exc) {
            trailer = true;
            rc = ((fi.total_samples != -1 && fi.out_frames != fi.total_samples) || r.crc_errors > 0) ? 1 : 0;
        }
    }
    // header: the stored RIFF header unless float, else RiffChunkHeader + "fmt " + WaveHeader + "data"
    // (WvDemo.cs:74-105, ChunkHeader.cs:29-45, RiffChunkHeader.cs:66-87, WaveHeader.cs:109-142)
    uint8_t synth[44];
    const uint8_t *hdr = nullptr;
    int64_t hlen = 0;
    if (fi.header_off >= 0 && !wi.is_float) {
        hdr = b->blob.data() + (size_t)(fi.blob_base + fi.header_off);
        hlen = fi.header_len;
    } else {
        memcpy(synth, "RIFF", 4);
        put_le32(synth + 4, (uint32_t)(total_native * block_align + 2 * 8 + 16) + 4);
        memcpy(synth + 8, "WAVE", 4);
        memcpy(synth + 12, "fmt ", 4);
        put_le32(synth + 16, 16);
        synth[20] = 1;
        synth[21] = 0;
        synth[22] = (uint8_t)nch;
        synth[23] = (uint8_t)(nch >> 8);
        put_le32(synth + 24, (uint32_t)wi.sample_rate);
        put_le32(synth + 28, (uint32_t)(wi.sample_rate * block_align));
        synth[32] = (uint8_t)block_align;
        synth[33] = (uint8_t)(block_align >> 8);
        synth[34] = (uint8_t)wi.bits_per_sample;
        synth[35] = (uint8_t)(wi.bits_per_sample >> 8);
        memcpy(synth + 36, "data", 4);
        put_le32(synth + 40, (uint32_t)(total_native * block_align));
        hdr = synth;
        hlen = 44;
    }
    const int64_t pcm = frames * block_align;
    const int64_t tlen = trailer && fi.trailer_off >= 0 ? fi.trailer_len : 0;
    const int64_t total = hlen + pcm + tlen;
    *wav_len = total;
    *exit_code = rc;
    if (!out) return WVG_OK;  // size query
    if (cap < total) return WVG_ERR_SPACE;
    memcpy(out, hdr, (size_t)hlen);
    if (pcm) {
        HIPCHK(c, hipMemcpyAsync(out + hlen, b->d_pcm + b->pcm_off[(size_t)file], (size_t)pcm, hipMemcpyDeviceToHost,
                                 b->stream));
        HIPCHK(c, hipStreamSynchronize(b->stream));
    }
    if (tlen) memcpy(out + hlen + pcm, b->blob.data() + (size_t)(fi.blob_base + fi.trailer_off), (size_t)tlen);
    return WVG_OK;
}

// ---------------------------------------------------------------------------
// Streaming WavpackUnpackSamples (WavPackUtils.cs:200-282): the caller's calls
// are served a window at a time.  The file is decoded on the device on the
// first call (the blocks are independent: one launch decodes them all, and
// 288 GB of HBM holds any file's int32 output); the host only ever holds the
// compressed file and two windows of `window` frames in page-locked staging,
// the next window's DMA running while the caller consumes the current one.
// crc_errors are counted as each block's last frame is handed out (:273-275),
// and the call that the reference throws in returns WVG_ERR_EXCEPTION after
// the calls before it returned their frames.
// ---------------------------------------------------------------------------
struct wvg_stream {
    wvg_ctx *ctx = nullptr;
    wvg_batch *b = nullptr;
    std::vector<uint8_t> file;
    uint32_t flags = 0;
    int64_t seek = -1;            // SetSample target (-1: none)
    int chunk = 0;                // the request size the decode was scheduled at (0: not decoded)
    int64_t window = 0;           // frames per staged window
    wvg_file_info info;
    wvg_file_result res;
    int nch = 1;
    bool throws = false;
    int schedule_changed = 0;
    int64_t pos = 0, limit = 0;   // frames handed out since the decode's start / before the end or the throw
    int64_t errors_before = 0;    // crc_errors of calls made before a SetSample
    int64_t index0 = 0;           // stream.sample_index when the decode's first call starts
    std::vector<int64_t> blk_end;
    std::vector<uint32_t> blk_st;
    size_t blk_next = 0;          // blocks counted so far (their last frame was handed out)
    int64_t errors = 0;
    PinnedBuf stage[2];
    int64_t lo[2] = {0, 0}, hi[2] = {0, 0};  // frames staged in stage[k] (hi == lo: none)
    hipEvent_t ev[2] = {nullptr, nullptr};
    int cur = 0;
    int broken = 0;               // a SetSample whose decode failed: every later call returns this code
};

static int stream_fetch(wvg_stream *s, int k, int64_t from) {
    wvg_ctx *c = s->ctx;
    const int64_t to = std::min(from + s->window, s->limit);
    s->lo[k] = from;
    s->hi[k] = to;
    if (to <= from) return WVG_OK;
    if (!s->stage[k].resize(sizeof(int32_t) * (size_t)((to - from) * s->nch))) return WVG_ERR_SPACE;
    const int32_t *src = s->b->d_out + s->info.out_offset + from * s->nch;
    HIPCHK(c, hipMemcpyAsync(s->stage[k].data(), src, sizeof(int32_t) * (size_t)((to - from) * s->nch),
                             hipMemcpyDeviceToHost, s->b->stream));
    HIPCHK(c, hipEventRecord(s->ev[k], s->b->stream));
    return WVG_OK;
}

// (re)decode the file with the calls scheduled at `chunk` frames
static int stream_decode(wvg_stream *s, int chunk) {
    wvg_ctx *c = s->ctx;
    HIPCHK(c, hipSetDevice(c->device));
    if (s->b && s->b->chunk != chunk) {
        wvg_batch_free(s->b);
        s->b = nullptr;
    }
    if (!s->b) {
        s->b = wvg_batch_new(c, chunk);
        if (!s->b) return WVG_ERR_HIP;
    } else {
        wvg_batch_reset(s->b);
    }
    wvg_batch *b = s->b;
    const int idx = s->seek >= 0 ? wvg_batch_add_file_at(b, s->file.data(), s->file.size(), s->flags, s->seek, &s->info)
                                 : wvg_batch_add_file(b, s->file.data(), s->file.size(), s->flags, &s->info);
    if (idx != 0) return idx < 0 ? idx : WVG_ERR_ARG;
    int rc = wvg_batch_upload(b);
    if (rc == WVG_OK) rc = wvg_batch_decode(b, nullptr);
    if (rc == WVG_OK) rc = wvg_batch_download(b, nullptr, 0);  // statuses only
    if (rc == WVG_OK) rc = wvg_batch_file_result(b, 0, &s->res);
    if (rc != WVG_OK) return rc;
    s->info.out_offset = b->infos[0].out_offset;
    s->nch = s->info.reduced_channels > 0 ? s->info.reduced_channels : 1;
    s->throws = s->res.exception != 0;
    s->limit = s->throws ? s->res.exception_frame : s->info.out_frames;
    s->blk_end.assign((size_t)s->res.num_blocks, 0);
    s->blk_st.assign((size_t)s->res.num_blocks, 0);
    if (s->res.num_blocks > 0) {
        rc = wvg_batch_file_blocks(b, 0, s->blk_end.data(), s->blk_st.data(), s->res.num_blocks);
        if (rc < 0) return rc;
    }
    s->blk_next = 0;
    s->errors = 0;
    s->pos = 0;
    s->index0 = s->info.sample_index0;
    s->chunk = chunk;
    s->lo[0] = s->hi[0] = s->lo[1] = s->hi[1] = 0;
    return stream_fetch(s, s->cur, 0);
}

static void stream_count_blocks(wvg_stream *s) {
    while (s->blk_next < s->blk_end.size() && s->blk_end[s->blk_next] <= s->pos) {
        if (s->blk_st[s->blk_next] & ST_CRC_ERROR) s->errors++;
        s->blk_next++;
    }
}

wvg_stream *wvg_stream_open(wvg_ctx *ctx, const uint8_t *file, size_t len, uint32_t open_flags, int64_t window_frames,
                            wvg_file_info *info) {
    if (!ctx || (!file && len)) return nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
    wvg_stream *s = new wvg_stream();
    s->ctx = ctx;
    s->file.assign(file, file + len);
    s->flags = open_flags;
    s->window = window_frames > 0 ? window_frames : ((int64_t)1 << 18);
    memset(&s->res, 0, sizeof(s->res));
    const int rc = wvg_probe_file(s->file.data(), s->file.size(), open_flags, SAMPLE_BUFFER_SIZE, &s->info);
    if (info) *info = s->info;
    if (rc != WVG_OK || hipEventCreateWithFlags(&s->ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev[1], hipEventDisableTiming) != hipSuccess) {
        wvg_stream_close(s);
        return nullptr;
    }
    s->index0 = s->info.sample_index0;
    return s;
}

void wvg_stream_close(wvg_stream *s) {
    if (!s) return;
    hipSetDevice(s->ctx->device);
    if (s->b) wvg_batch_free(s->b);  // waits for the staged DMAs on its stream
    for (auto &e : s->ev)
        if (e) hipEventDestroy(e);
    delete s;
}

int64_t wvg_stream_unpack(wvg_stream *s, int32_t *buffer, int64_t samples) {
    if (!s || samples < 0 || (!buffer && samples)) return WVG_ERR_ARG;
    if (s->broken) return s->broken;
    if (samples > INT32_MAX) return WVG_ERR_ARG;
    if (!s->chunk || ((int)samples != s->chunk && s->pos == 0 && samples > 0)) {
        // the first call (or a new request size before any frame went out): the decode is
        // scheduled at this request size, as the reference's seams follow the caller's calls
        const int rc = stream_decode(s, samples > 0 ? (int)samples : SAMPLE_BUFFER_SIZE);
        if (rc != WVG_OK) return rc;
    } else if ((int)samples != s->chunk) {
        s->schedule_changed = 1;  // later calls of another size: served from the first schedule
    }
    if (s->pos >= s->limit) return s->throws ? WVG_ERR_EXCEPTION : 0;
    int64_t n = std::min(samples, s->limit - s->pos);
    // a call the reference ends early (its loop breaks on a header / unpack_init failure).
    // The cuts are output positions: a break falls where a block's header or unpack_init
    // fails, whatever the request size, so they hold after the caller changes its size too
    // (schedule_changed); the file-end cut is the limit itself.  What a size change can
    // move is a break landing exactly on a call boundary, which returns 0 frames (the end
    // of a WvDemo-style loop) under one schedule and a short call under another -- such a
    // stream is served from its first schedule, and wvg_stream_state reports it.
    const std::vector<int64_t> &cuts = s->b->finfo[0].call_cuts;
    auto cut = std::upper_bound(cuts.begin(), cuts.end(), s->pos);
    if (cut != cuts.end() && *cut - s->pos < n) n = *cut - s->pos;
    wvg_ctx *c = s->ctx;
    int64_t done = 0;
    while (done < n) {
        const int64_t f = s->pos + done;
        int k = s->cur;
        if (!(f >= s->lo[k] && f < s->hi[k])) {
            k ^= 1;
            if (!(f >= s->lo[k] && f < s->hi[k])) {  // not staged (the first call, or a skipped window)
                const int rc = stream_fetch(s, k, f);
                if (rc != WVG_OK) return rc;
            }
            s->cur = k;
            // the next window's DMA runs while this one is served
            const int rc = stream_fetch(s, k ^ 1, s->hi[k]);
            if (rc != WVG_OK) return rc;
        }
        HIPCHK(c, hipEventSynchronize(s->ev[k]));
        const int64_t m = std::min(n - done, s->hi[k] - f);
        memcpy(buffer + done * s->nch, s->stage[k].data() + sizeof(int32_t) * (size_t)((f - s->lo[k]) * s->nch),
               sizeof(int32_t) * (size_t)(m * s->nch));
        done += m;
    }
    s->pos += n;
    stream_count_blocks(s);
    return n;
}

int wvg_stream_set_sample(wvg_stream *s, int64_t sample) {
    if (!s || sample < 0) return WVG_ERR_ARG;
    if (s->broken) return s->broken;
    // the block search runs on the host framing (WavPackUtils.cs:521-594)
    FramingOutput fo;
    FileInfo fi;
    frame_file(s->file.data(), s->file.size(), 0, 0, s->flags, s->chunk ? s->chunk : SAMPLE_BUFFER_SIZE, fo, fi,
               sample);
    if (!fi.open_ok) return 0;
    if (fi.seek_result < 0) return WVG_ERR_EXCEPTION;
    if (fi.seek_result == 0) return 0;
    // the new seek and error count are committed only once its decode succeeded
    const int64_t before = s->errors_before + s->errors, prev_seek = s->seek;
    s->seek = sample;
    // decode now: the discard calls' block ends count towards the errors at once
    const int rc = stream_decode(s, s->chunk ? s->chunk : SAMPLE_BUFFER_SIZE);
    if (rc != WVG_OK) {
        // s->info and s->b may already belong to the new decode: nothing may be served
        // from mixed state, so the stream is invalid from here on
        s->seek = prev_seek;
        s->chunk = 0;
        s->pos = s->limit = 0;
        s->lo[0] = s->hi[0] = s->lo[1] = s->hi[1] = 0;
        s->broken = rc;
        return rc;
    }
    s->errors_before = before;  // (the index is where the decode's first call starts: info.sample_index0)
    stream_count_blocks(s);
    return 1;
}

int wvg_stream_state(const wvg_stream *s, int64_t *sample_index, int64_t *crc_errors, int32_t *lossy,
                     int32_t *schedule_changed) {
    if (!s) return WVG_ERR_ARG;
    if (sample_index) *sample_index = s->chunk ? s->index0 + s->pos : s->info.sample_index0;
    if (crc_errors) *crc_errors = s->errors_before + s->errors;
    if (lossy) *lossy = s->chunk ? s->res.lossy : s->info.lossy;
    if (schedule_changed) *schedule_changed = s->schedule_changed;
    return WVG_OK;
}

}  // extern "C"
