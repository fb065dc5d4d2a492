/*
 * wv_oracle.h -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * A plain-C, line-by-line restatement of the reference C# WavPack decoder
 * (Quake4/WavPackDecoder, /root/reference).  It exists so that tests/ can check
 * the HIP decode path bit-exactly and so bench.py can time the reference
 * algorithm on the host ("cpu_baseline", kind "port").  Nothing in the product
 * path (wavpackdecoder_amd/) may link, load or call it.
 *
 * The reference is C# (.NET 3.5, WavPack.Decoder.csproj:24); there is no
 * dotnet/mono in this image, so it cannot be built or run here and no
 * oracle/_ref exists.  The reference ships no golden vectors either, so this
 * oracle is pinned by (a) lossless round trips against the repo's own encoder
 * (external truth for every lossless integer mode), (b) the per-block CRC the
 * format embeds, and (c) hand-derived known answers for the table functions
 * (tests/test_oracle_kat.py).  For hybrid/float/DSD-coded modes parity is
 * oracle-vs-GPU only ("parity unpinned" beyond the CRC), see DESIGN.md.
 *
 * C# semantics reproduced: wrapping int32 arithmetic
 * (built with -fwrapv), masked shift counts, (short) weight stores, sticky
 * cross-block state, the 0xFF past-end fill, and C# exceptions
 * (IndexOutOfRange / DivideByZero) which are modelled as an "exception" status.
 */
#ifndef WV_ORACLE_H
#define WV_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wvo_ctx wvo_ctx;

/* WavPackUtils.WavpackOpenFileInput (WavPackUtils.cs:36-120) over an in-memory
 * file.  The bytes must stay alive while the context is used.  Never returns
 * NULL (like the C#); check wvo_get_error_message(). */
wvo_ctx *wvo_open(const uint8_t *file, size_t len, uint32_t flags);
void wvo_close(wvo_ctx *ctx);

/* WavPackUtils.WavpackUnpackSamples (WavPackUtils.cs:200-282).
 * buffer_len is the C# int[] Length (bounds are checked as C# would).
 * Returns frames unpacked; -1 if a C# exception escaped (see wvo_exception). */
int64_t wvo_unpack_samples(wvo_ctx *ctx, int32_t *buffer, int64_t buffer_len, int64_t samples);

/* WavPackUtils.WavpackFormatSamples (WavPackUtils.cs:288-341). Returns 1/0. */
int wvo_format_samples(const int32_t *src, int64_t samcnt, int bps, uint8_t *pcm,
                       int64_t pcm_len, int offset, int dsd);

/* getters (WavPackUtils.cs:346-499) */
int64_t wvo_get_num_samples(wvo_ctx *ctx, int native);
int64_t wvo_get_sample_index(wvo_ctx *ctx);
int64_t wvo_get_num_errors(wvo_ctx *ctx);
int wvo_lossy(wvo_ctx *ctx);
int64_t wvo_get_sample_rate(wvo_ctx *ctx);
int wvo_get_num_channels(wvo_ctx *ctx);
int wvo_get_bits_per_sample(wvo_ctx *ctx);
int wvo_get_bytes_per_sample(wvo_ctx *ctx);
int wvo_get_reduced_channels(wvo_ctx *ctx);
int wvo_get_mode(wvo_ctx *ctx);
int wvo_get_version(wvo_ctx *ctx);
int wvo_get_is_float(wvo_ctx *ctx);
int wvo_get_is_five(wvo_ctx *ctx);
int wvo_get_file_format(wvo_ctx *ctx);
const char *wvo_get_error_message(wvo_ctx *ctx);
int wvo_exception(wvo_ctx *ctx); /* 0 none, else WVO_EXC_* */
const uint8_t *wvo_get_header(wvo_ctx *ctx, int *len);
const uint8_t *wvo_get_trailer(wvo_ctx *ctx, int *len);

enum { WVO_EXC_NONE = 0, WVO_EXC_INDEX = 1, WVO_EXC_DIVZERO = 2, WVO_EXC_IO = 3, WVO_EXC_STACK = 4, WVO_EXC_HANG = 5 };

/* WavPackUtils.SetSample -> seek (WavPackUtils.cs:509-594): 1 positioned (the C#
 * `true`), 0 not (`false`), -1 an exception escaped (or the discard loop would
 * never end: WVO_EXC_HANG). */
int wvo_set_sample(wvo_ctx *ctx, int64_t sample);

/* open + SetSample(start) + WavpackUnpackSamples loop of `chunk` frames per call
 * (like wvo_decode_file); *seek_rc receives wvo_set_sample's result.
 * Returns frames after the seek, -2 open error, -3 exception. */
int64_t wvo_decode_file_from(const uint8_t *file, size_t len, int64_t start, int32_t *out, int64_t out_cap, int chunk,
                             int64_t *crc_errors, int *nch, int *seek_rc);

/* Convenience used by tests/bench: open + loop WavpackUnpackSamples with
 * `chunk` frames per call exactly like WvDemo.cs:110-135 (chunk 4096), all
 * output concatenated into out (capacity out_cap int32 values).
 * Returns total frames unpacked, or a negative value on open error (-2) or
 * exception (-3).  *crc_errors, *lossy, *nch receive the context values. */
int64_t wvo_decode_file(const uint8_t *file, size_t len, int32_t *out, int64_t out_cap,
                        int chunk, int64_t *crc_errors, int *lossy, int *nch);

/* WvDemo.Main equivalent (WvDemo.cs:15-168) producing the .wav bytes in memory.
 * Returns the C# exit code (0/1). *wav (malloc'd, caller frees) and *wav_len
 * receive what WvDemo would have written before returning. */
int wvo_demo(const uint8_t *file, size_t len, uint8_t **wav, size_t *wav_len);
void wvo_free(void *p);

/* Table functions exported for known-answer tests (WordsUtils.cs:513-661). */
int wvo_exp2s(int log);
int wvo_mylog2(int64_t avalue);
int wvo_log2s(int value);
int wvo_count_bits(int64_t av);
int wvo_restore_weight(int8_t weight);
/* read_code over a raw byte buffer starting at bit 0: returns the code, and the
 * number of bits consumed in *used (BitsUtils.cs + WordsUtils.cs:546-570). */
int64_t wvo_read_code_bytes(const uint8_t *bytes, int len, int64_t maxcode, int *used);

#ifdef __cplusplus
}
#endif
#endif
