/*
 * wvgpu.h -- C-ABI of the MI355X WavPack block-decode path (libwvgpu.so).
 *
 * Drop-in boundary for the reference's hot path
 *   public static long WavPackUtils.WavpackUnpackSamples(WavpackContext wpc, int[] buffer, long samples)
 *   (Quake4/WavPackDecoder WavPackUtils.cs:200-282)
 * and the calls around it that a C# host needs to keep its API:
 *   WavpackOpenFileInput   WavPackUtils.cs:36-120   -> wvg_batch_add_file (framing, info)
 *   WavpackUnpackSamples   WavPackUtils.cs:200-282  -> wvg_batch_decode (+ download)
 *   WavpackFormatSamples   WavPackUtils.cs:288-341  -> wvg_format_samples
 *   WavpackGetNumErrors    WavPackUtils.cs:363      -> wvg_file_result.crc_errors
 *   WavpackLossy           WavPackUtils.cs:371      -> wvg_file_result.lossy
 *   other getters          WavPackUtils.cs:346-499  -> wvg_file_info
 *
 * Blittable types only (P/Invoke ready): every buffer is caller-owned; the
 * library keeps device copies owned by the batch handle.  Errors are int
 * return codes (0 = OK, < 0 = error) plus wvg_last_error(); no C++
 * exception crosses the ABI.  One context per device per host thread.
 *
 * Output contract: a batch decodes every file exactly as a caller looping
 * WavpackUnpackSamples(wpc, buffer, chunk_frames) (WvDemo.cs:110-135) would
 * receive it, concatenated: int32 per channel-sample, interleaved,
 * right-justified; float files as clipped 24-bit ints (FloatUtils.cs:32-56);
 * DSD as one byte value per channel-sample.
 */
#ifndef WVGPU_H
#define WVGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WVG_OK 0
#define WVG_ERR_HIP (-1)      /* HIP runtime error (see wvg_last_error) */
#define WVG_ERR_ARG (-2)      /* bad argument / state */
#define WVG_ERR_OPEN (-3)     /* WavpackOpenFileInput failed (info.error holds the message) */
#define WVG_ERR_SPACE (-4)    /* caller buffer too small */
#define WVG_ERR_TIMEOUT (-5)  /* a kernel's bounded wait ran out (a decoder bug, never a property of the stream) */
#define WVG_ERR_EXCEPTION (-6) /* wvg_stream_*: the reference raises a C# exception in this call */

/* per-block status bits (wvg_file_result.status_or) */
#define WVG_ST_CRC_CHECKED 0x01u
#define WVG_ST_CRC_ERROR 0x02u
#define WVG_ST_MUTED 0x04u
#define WVG_ST_BITS_ERROR 0x08u
#define WVG_ST_EXCEPTION 0x10u   /* the reference raises a C# exception in this block */
#define WVG_ST_UNSUPPORTED 0x20u /* depends on decode state of an earlier block (never in well-formed files) */
#define WVG_ST_DSD_MUTE 0x40u
#define WVG_ST_NONDET 0x80u      /* reference output depends on stale caller-buffer contents */
#define WVG_ST_TIMEOUT 0x100u    /* the parser/reconstruction handshake timed out: output invalid (not a reference outcome) */
#define WVG_ST_REDONE 0x200u     /* wvg_batch_block_status only: the lane kernel handed this block back and the
                                    one-workgroup-per-block kernel decoded it (a cost, never a result: masked out
                                    of wvg_file_result.status_or) */
#define WVG_ST_UNWRITTEN 0x40000000u /* wvg_batch_block_status only: no decode has stored this block's status since
                                        wvg_batch_poison (a bench/test check that a decode really ran) */

typedef struct wvg_ctx wvg_ctx;
typedef struct wvg_batch wvg_batch;

/* What WavpackOpenFileInput + the getters report (WavPackUtils.cs:36-120, 346-499). */
typedef struct {
    int32_t open_ok;            /* 0 => error[] holds wpc.error_message */
    int32_t num_channels;       /* WavpackGetNumChannels */
    int32_t reduced_channels;   /* WavpackGetReducedChannels (ints per output frame) */
    int32_t bits_per_sample;    /* WavpackGetBitsPerSample (DSD: /8 applied like the getter) */
    int32_t bytes_per_sample;   /* WavpackGetBytesPerSample */
    int32_t version;            /* WavpackGetVersion */
    int32_t mode;               /* WavpackGetMode */
    int32_t is_float;           /* WavpackGetIsFloat */
    int32_t is_five;            /* WavpackGetIsFive */
    int32_t file_format;        /* WavpackGetFileFormat */
    int32_t lossy;              /* WavpackLossy at open */
    uint32_t dsd_multiplier;
    int64_t sample_rate;        /* WavpackGetSampleRate */
    int64_t total_samples;      /* WavpackGetNumSamples(native=false), -1 unknown */
    int64_t out_frames;         /* frames the chunked caller receives */
    int64_t out_offset;         /* int32 index of this file's output inside the batch */
    int64_t header_off, header_len;   /* RIFF/ALT header bytes inside the file (WavpackGetHeader), -1 none */
    int64_t trailer_off, trailer_len; /* WavpackGetTrailer */
    char error[96];
    int32_t seek_result;        /* wvg_batch_add_file_at: SetSample's result (1 true, 0 false, -1 it threw) */
    int32_t reserved;
    int64_t sample_index0;      /* WavpackGetSampleIndex when the first WavpackUnpackSamples call starts
                                   (after SetSample: the target); it then advances by the frames returned */
} wvg_file_info;

typedef struct {
    int64_t frames;             /* == info.out_frames unless an exception stopped the decode */
    int64_t crc_errors;         /* WavpackGetNumErrors after the last call */
    int32_t lossy;              /* WavpackLossy after the last call */
    int32_t exception;          /* the reference would have thrown (WvDemo exits 1) */
    uint32_t status_or;         /* OR of the WVG_ST_* bits of all blocks */
    int32_t num_blocks;
    int64_t exception_frame;    /* with exception: frames the calls before the throwing call returned
                                   (the throwing call is the one that starts there); -1 otherwise */
} wvg_file_result;

/* Device + stream ownership.  device < 0 => current device. */
wvg_ctx *wvg_open(int device);
void wvg_close(wvg_ctx *ctx);
const char *wvg_last_error(wvg_ctx *ctx);

/* A batch of files decoded together.  chunk_frames is the caller's per-call
 * frame count (Defines.SAMPLE_BUFFER_SIZE = 4096 for WvDemo); it fixes the
 * reference's chunk seams (weight (short) stores, mute granularity). */
wvg_batch *wvg_batch_new(wvg_ctx *ctx, int chunk_frames);
void wvg_batch_free(wvg_batch *b);

/* Frame one file (host): parses headers/metadata, records the blocks.
 * The bytes are copied into the batch.  Returns the file index (>= 0) or
 * WVG_ERR_OPEN (info->error set; the file contributes no output). */
int wvg_batch_add_file(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, wvg_file_info *info);

/* n files at once, framed on `threads` host threads (<= 0: WVG_FRAME_THREADS or
 * the hardware concurrency, at most 16); the same result as n wvg_batch_add_file
 * calls in order.  indices[i] receives file i's index or WVG_ERR_OPEN; returns n. */
int wvg_batch_add_files(wvg_batch *b, int n, const uint8_t *const *files, const size_t *lens, uint32_t open_flags,
                        int threads, wvg_file_info *infos, int32_t *indices);

/* The same, for a caller that calls WavPackUtils.SetSample(wpc, start_sample)
 * (WavPackUtils.cs:509-594: the block search, then decode-and-discard up to the
 * sample in calls of 4096 / reduced-channels frames) right after opening: the
 * file's output is what the following WavpackUnpackSamples calls return.
 * info->seek_result holds SetSample's result; when it is 0 the output starts
 * at the beginning, as the reference's context does. */
int wvg_batch_add_file_at(wvg_batch *b, const uint8_t *file, size_t len, uint32_t open_flags, int64_t start_sample,
                          wvg_file_info *info);

/* open_flags bit beyond the reference (whose only flag is OPEN_2CH_MAX = 0x8,
 * Defines.cs:26): FLOAT_DATA blocks decode to IEEE-754 float32 bit patterns by
 * WavPack 4's float_values -- exact when the block carries its classic
 * ID_WVX_BITSTREAM (in the .wv, or in the .wvc for a hybrid file) -- instead of
 * FloatUtils.cs:32-56's scaling to 24-bit integers.  Blocks with a wvx stream
 * check its crc (WVG_ST_CRC_ERROR); a NEW-format float wvx stream is
 * WVG_ST_UNSUPPORTED.  Parity: round trip to the encoder's float input. */
#define WVG_OPEN_EXACT_FLOAT 0x40000000u

/* A hybrid .wv file with its .wvc correction file: the hybrid blocks decode
 * EXACTLY (lossless) instead of the reference's lossy output.  Beyond the
 * reference (it opens ID_WVC_BITSTREAM, UnpackUtils.cs:96-106, but never reads
 * it): parity is the round trip to the encoder's input.  Returns the
 * file index or WVG_ERR_OPEN, as wvg_batch_add_file. */
int wvg_batch_add_file_wvc(wvg_batch *b, const uint8_t *file, size_t len, const uint8_t *wvc, size_t wvc_len,
                           uint32_t open_flags, wvg_file_info *info);

/* n files framed ON THE DEVICE at the next wvg_batch_upload (the
 * WavpackOpenFileInput header + sub-block walk of WavPackUtils.cs:36-120,600-671,
 * UnpackUtils.cs:24-68, MetadataUtils.cs:15-192 as kernels, open_flags 0).  The
 * bytes are copied now and file slots reserved (indices[i]); a file outside the
 * device framer's scope (DSD mode 1, wvx, sticky state, junk, damaged headers) is framed
 * by the host at the same upload with the same result as wvg_batch_add_file.
 * The files' infos are available after the upload (wvg_batch_file_info). */
int wvg_batch_add_files_device(wvg_batch *b, int n, const uint8_t *const *files, const size_t *lens,
                               int32_t *indices);
/* A file's info (after the upload for device-framed files); WVG_ERR_OPEN if it did not open. */
int wvg_batch_file_info(const wvg_batch *b, int file, wvg_file_info *info);
/* Files [first, first + n) at once (one call for a whole device-framed slice); returns how
 * many were copied (fewer when the batch has fewer files). */
int wvg_batch_file_infos(const wvg_batch *b, int first, int n, wvg_file_info *infos);
/* Files of the batch framed on the device / by the host fallback at its uploads. */
int wvg_batch_framing_stats(const wvg_batch *b, int64_t *device_files, int64_t *host_files);
/* Diagnostics: which launch groups the last wvg_batch_decode ran on the lane / row
 * kernels (bit t: PCM term-set group t, 0..7; bit 8: .wvc blocks; bit 9: DSD mode 3;
 * bit 10: DSD mode 1) -- under WVG_KERNEL_AUTO the choice depends on whether other
 * batches of the context overlapped within the last second.  No reference counterpart. */
int wvg_batch_lane_groups(const wvg_batch *b, uint32_t *mask);

/* Drop every file of the batch but keep its device and page-locked host
 * buffers (a decode server refills one batch per request). */
int wvg_batch_reset(wvg_batch *b);

/* Copy blob + descriptors to the device and zero the output (device buffers are
 * kept across uploads of a refilled batch and only grown). */
int wvg_batch_upload(wvg_batch *b);

/* Enqueue the decode kernels on `stream` (hipStream_t, NULL = the batch's own
 * stream).  Input and output stay in HBM.  Every batch owns its streams, so
 * batches decode concurrently; nothing synchronises the whole device. */
int wvg_batch_decode(wvg_batch *b, void *stream);
/* Wait for the batch's last decode / format (an event on the stream it ran on). */
int wvg_batch_sync(wvg_batch *b);
/* Which kernel decodes the batch's lossless PCM blocks whose decorr list has a
 * compile-time specialisation (no reference counterpart: a scheduling choice).
 * WVG_KERNEL_LANE: one lane per block, 64 blocks per workgroup -- one SIMD issue
 * slot moves 64 blocks, so batches in flight decode many times more per second --
 * for lossless PCM blocks, hybrid stereo blocks of WavPack's default list and DSD
 * mode-3 blocks; blocks a lane cannot follow exactly are decoded again by the
 * two-wave kernel (the pipelined kernel for WavPack's 16-term 'high' list, the
 * wave-per-block kernel for DSD) within the same decode.  WVG_KERNEL_TWO_WAVE: one
 * workgroup per block (a scalar parser wave and a reconstruction wave; one wave
 * per DSD block), the lowest latency for a batch alone.  WVG_KERNEL_AUTO (the
 * default): the lane kernels once the context has had a decode issued while another
 * of its batches was running; until then (one batch at a time) the two-wave /
 * wave-per-block kernels for launch groups of at most 2,048 blocks (larger ones on
 * lanes).  A decode issued while other batches
 * run also keeps all its launch groups on its own stream (streams share the
 * process's few hardware queues).  Results are identical in every mode
 * (WVG_LANE_KERNEL=0/1 in the environment fixes the kernel for new batches). */
#define WVG_KERNEL_TWO_WAVE 0
#define WVG_KERNEL_LANE 1
#define WVG_KERNEL_AUTO 2
int wvg_batch_set_kernel(wvg_batch *b, int kernel);
void *wvg_batch_stream(wvg_batch *b);  /* the batch's own hipStream_t */
/* Verification aid (no reference counterpart): overwrite the uploaded batch's int32
 * output with `byte` in every byte and mark every decodable block WVG_ST_UNWRITTEN, so
 * that what a download shows afterwards was written by the decodes issued after this
 * call.  Waits for the batch's earlier work.  (Gaps the reference zero-fills are left
 * poisoned until the next wvg_batch_upload.) */
int wvg_batch_poison(wvg_batch *b, int byte);
/* Device timing of every following decode (an event pair around each launch, on its
 * stream); wvg_batch_timed waits for them and returns the mean and the count. */
int wvg_batch_set_timing(wvg_batch *b, int on);
int wvg_batch_timed(wvg_batch *b, float *avg_ms, int *count);
/* With timing on: for the last decode, the time from its start to the end of
 * each launch group on its own stream, ms[g] for g = term set 0..7, 8 generic
 * PCM, 9 DSD, 10 DSD mode 1 (-1: not launched); cap >= 11. */
int wvg_batch_group_times(wvg_batch *b, float *ms, int cap);

int64_t wvg_batch_out_ints(const wvg_batch *b);
int32_t *wvg_batch_device_out(wvg_batch *b);      /* device pointer to the int32 output */
int64_t wvg_batch_num_blocks(const wvg_batch *b);
int64_t wvg_batch_bytes_in(const wvg_batch *b);   /* compressed bytes of all decoded blocks */
int64_t wvg_batch_frames(const wvg_batch *b);     /* frames of all decoded blocks */

/* Download output (and per-block statuses) and fill per-file results.
 * host_out == NULL with cap_ints == -1: into the batch's own page-locked
 * buffer (full PCIe rate), read through wvg_batch_host_out until the next
 * download or wvg_batch_free; host_out == NULL otherwise: statuses only. */
int wvg_batch_download(wvg_batch *b, int32_t *host_out, int64_t cap_ints);
int32_t *wvg_batch_host_out(wvg_batch *b);
int wvg_batch_file_result(wvg_batch *b, int file, wvg_file_result *res);
/* per-block status words (after download), one per decoded block in file order */
int wvg_batch_block_status(wvg_batch *b, uint32_t *out, int64_t cap);
/* Diagnostics (a library built with -DWV_LANE_COUNTERS=1 -- make counters -- and
 * batches created with WVG_LANE_COUNTERS=1 in the environment; zeros otherwise): per
 * parser wave of term set `ts`'s last lane-kernel decode, 16 words -- cycles, groups,
 * then groups taken as a zero-run bulk step / no-run words / split no-run words /
 * run-aware words / checked words at once / checked replay, then the cycles spent
 * waiting for the reconstruction wave and for the payload loads, in the groups'
 * words and in their ring stores (low 32 bits of each count).  Returns the wave
 * count (out needs 16 per wave), WVG_ERR_ARG without counters. */
int wvg_batch_lane_counters(wvg_batch *b, int ts, uint32_t *out, int64_t cap);
/* The blocks of one file (after download): for block k, end_frame[k] = the number of
 * frames the caller has received when the block's last frame is unpacked (that is
 * when WavpackUnpackSamples runs check_crc_error, WavPackUtils.cs:273-275), and its
 * status word.  Returns the block count, or < 0. */
int wvg_batch_file_blocks(wvg_batch *b, int file, int64_t *end_frame, uint32_t *status, int64_t cap);

/* Device-side timing of `iters` back-to-back decodes (hipEvents on the
 * batch stream).  *ms receives the average per decode. */
int wvg_batch_time(wvg_batch *b, int iters, float *ms);

/* One-shot convenience: frame + upload + decode + download one file. */
int wvg_decode_file(wvg_ctx *ctx, const uint8_t *file, size_t len, int chunk_frames, int32_t *out, int64_t cap_ints,
                    wvg_file_info *info, wvg_file_result *res);

/* WavpackOpenFileInput (WavPackUtils.cs:36-120) without a device: host framing
 * only, fills what the getters report.  WVG_ERR_OPEN when the file does not open. */
int wvg_probe_file(const uint8_t *file, size_t len, uint32_t open_flags, int chunk_frames, wvg_file_info *info);

/* WavpackFormatSamples (WavPackUtils.cs:288-341) on the host: int32 -> LE PCM bytes. */
int wvg_format_samples(const int32_t *src, int64_t samcnt, int bps, uint8_t *pcm, int64_t pcm_len, int offset,
                       int dsd);

/* WavpackFormatSamples over a decoded batch, on the device (epilogue kernel on
 * `stream` after wvg_batch_decode): every file's int32 output becomes its
 * little-endian PCM image at info.bytes_per_sample, 1-byte samples +128 unless
 * `dsd` (the reference's dsd argument; WvDemo.cs:125 passes false).  The image
 * stays in HBM; file i starts at byte wvg_batch_pcm_offset(b, i). */
int wvg_batch_format(wvg_batch *b, int dsd, void *stream);
int64_t wvg_batch_pcm_bytes(const wvg_batch *b);
int64_t wvg_batch_pcm_offset(const wvg_batch *b, int file);  /* -1: the file did not open */
uint8_t *wvg_batch_device_pcm(wvg_batch *b);                 /* device pointer to the PCM image */
/* host == NULL and cap == -1: into the batch's page-locked buffer (full PCIe
 * rate), read through wvg_batch_host_pcm until the next such download. */
int wvg_batch_download_pcm(wvg_batch *b, uint8_t *host, int64_t cap);
uint8_t *wvg_batch_host_pcm(wvg_batch *b);
/* The same download into the batch's page-locked buffer, queued behind the format
 * on the batch stream without waiting for it: a decode server issues a request's
 * upload, decode, format and download back to back and takes the PCM
 * (wvg_batch_host_pcm) after wvg_batch_sync -- the next reset/upload of the batch
 * waits for it too.  (The reference's WavpackUnpackSamples + WavpackFormatSamples
 * calls, WavPackUtils.cs:200-341, return the PCM synchronously; this is their
 * batched, overlapped form.) */
int wvg_batch_download_pcm_async(wvg_batch *b);

/* WvDemo.Main (WvDemo.cs:15-168) for one file of a formatted batch built with
 * chunk_frames 4096: the .wav bytes it writes (stored RIFF header or the
 * synthesized RIFF/fmt/data headers, the PCM, the stored trailer) and its exit
 * code.  out == NULL queries the length only. */
int wvg_batch_wav(wvg_batch *b, int file, uint8_t *out, int64_t cap, int64_t *wav_len, int32_t *exit_code);

/* ---- Streaming WavpackUnpackSamples (WavPackUtils.cs:200-282) --------------
 * One file opened like WavpackOpenFileInput (WavPackUtils.cs:36-120; NULL when
 * it does not open -- info->error holds the message), then served call by call.
 * The first wvg_stream_unpack decodes the file on the device, its calls
 * scheduled at that call's `samples` (the reference's seams follow the caller's
 * request size; a different size before any frame went out re-decodes, a later
 * one is served from the first schedule and flagged).  Host memory holds the
 * compressed file and two staged windows of `window_frames` frames (0: 262,144);
 * the int32 output stays in HBM.  wvg_stream_unpack returns the frames written
 * to `buffer` (samples x reduced channels ints), 0 at the end, or
 * WVG_ERR_EXCEPTION on the call the reference throws in (the calls before it
 * returned their frames).  wvg_stream_set_sample is SetSample
 * (WavPackUtils.cs:509-594): 1, 0 (false) or WVG_ERR_EXCEPTION.
 * wvg_stream_state: WavpackGetSampleIndex (:355-358), WavpackGetNumErrors
 * (:363-366, counted as each block's last frame is handed out, :273-275),
 * WavpackLossy (:371-374). */
typedef struct wvg_stream wvg_stream;
wvg_stream *wvg_stream_open(wvg_ctx *ctx, const uint8_t *file, size_t len, uint32_t open_flags, int64_t window_frames,
                            wvg_file_info *info);
int64_t wvg_stream_unpack(wvg_stream *s, int32_t *buffer, int64_t samples);
int wvg_stream_set_sample(wvg_stream *s, int64_t sample);
int wvg_stream_state(const wvg_stream *s, int64_t *sample_index, int64_t *crc_errors, int32_t *lossy,
                     int32_t *schedule_changed);
void wvg_stream_close(wvg_stream *s);

#ifdef __cplusplus
}
#endif
#endif
