/*
 * wv_oracle.c -- TEST INFRASTRUCTURE ONLY.  Plain-C restatement of the
 * reference C# decoder (Quake4/WavPackDecoder) used as the parity oracle and
 * as the bench's CPU baseline ("port").  See wv_oracle.h for the contract.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 *
 * Every function cites the reference file:line it restates.  Build with
 * -fwrapv: C# int arithmetic wraps (unchecked is the csproj default).
 */
#include "wv_oracle.h"

#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Defines.cs:13-156                                                   */
/* ------------------------------------------------------------------ */
#define SAMPLE_BUFFER_SIZE 4096
#define BITSTREAM_BUFFER_SIZE (16 * 1024)
#define OPEN_2CH_MAX 0x8
#define BYTES_STORED 3
#define MONO_FLAG 4
#define HYBRID_FLAG 8
#define FALSE_STEREO 0x40000000
#define MONO_DATA (MONO_FLAG | FALSE_STEREO)
#define DSD_FLAG 0x80000000u
#define SHIFT_LSB 13
#define SHIFT_MASK (0x1fL << SHIFT_LSB)
#define FLOAT_DATA 0x80
#define SRATE_LSB 23
#define SRATE_MASK (0xfL << SRATE_LSB)
#define FINAL_BLOCK 0x1000
#define MIN_STREAM_VERS 0x402
#define MAX_STREAM_VERS 0x410
#define ID_OPTIONAL_DATA 0x20
#define ID_ODD_SIZE 0x40
#define ID_LARGE 0x80
#define ID_DUMMY 0x0
#define ID_DECORR_TERMS 0x2
#define ID_DECORR_WEIGHTS 0x3
#define ID_DECORR_SAMPLES 0x4
#define ID_ENTROPY_VARS 0x5
#define ID_HYBRID_PROFILE 0x6
#define ID_SHAPING_WEIGHTS 0x7
#define ID_FLOAT_INFO 0x8
#define ID_INT32_INFO 0x9
#define ID_WV_BITSTREAM 0xa
#define ID_WVC_BITSTREAM 0xb
#define ID_WVX_BITSTREAM 0xc
#define ID_CHANNEL_INFO 0xd
#define ID_DSD_BLOCK 0xe
#define ID_RIFF_HEADER (ID_OPTIONAL_DATA | 0x1)
#define ID_RIFF_TRAILER (ID_OPTIONAL_DATA | 0x2)
#define ID_ALT_HEADER (ID_OPTIONAL_DATA | 0x3)
#define ID_ALT_TRAILER (ID_OPTIONAL_DATA | 0x4)
#define ID_CONFIG_BLOCK (ID_OPTIONAL_DATA | 0x5)
#define ID_SAMPLE_RATE (ID_OPTIONAL_DATA | 0x7)
#define ID_ALT_EXTENSION (ID_OPTIONAL_DATA | 0x8)
#define ID_NEW_CONFIG_BLOCK (ID_OPTIONAL_DATA | 0xa)
#define ID_WVX_NEW_BITSTREAM (ID_OPTIONAL_DATA | ID_WVX_BITSTREAM)
#define ID_BLOCK_CHECKSUM (ID_OPTIONAL_DATA | 0xf)
#define JOINT_STEREO 0x10
#define INT32_DATA 0x100
#define HYBRID_BITRATE 0x200
#define HYBRID_BALANCE 0x400
#define INITIAL_BLOCK 0x800
#define FLOAT_SHIFT_SENT 4
#define FLOAT_ZEROS_SENT 8
#define FLOAT_SHIFT_SAME 2
#define FLOAT_EXCEPTIONS 0x20
#define MAX_NTERMS 16
#define MAX_TERM 8
#define MAG_LSB 18
#define MAG_MASK (0x1fL << MAG_LSB)
#define CONFIG_HYBRID_FLAG 8
#define CONFIG_FLOAT_DATA 0x80
#define CONFIG_FAST_FLAG 0x200
#define CONFIG_HIGH_FLAG 0x800
#define CONFIG_VERY_HIGH_FLAG 0x1000
#define CONFIG_LOSSY_MODE 0x1000000
#define CONFIG_EXTRA_MODE 0x2000000
#define MODE_LOSSLESS 0x2
#define MODE_HYBRID 0x4
#define MODE_FLOAT 0x8
#define MODE_HIGH 0x20
#define MODE_FAST 0x40
#define MODE_EXTRA 0x80
#define MODE_VERY_HIGH 0x400
#define MODE_XMODE 0x7000
#define MODE_DSD 0x10000

/* ------------------------------------------------------------------ */
/* C# runtime emulation: exceptions, checked array access, shifts      */
/* ------------------------------------------------------------------ */
static __thread jmp_buf *g_jmp;
static __thread int g_exc;

static void cs_throw(int kind) {
    g_exc = kind;
    longjmp(*g_jmp, 1);
}

/* C# `int << n` / `int >> n` mask the count with 31, `long` with 63. */
static inline int32_t shl32(int32_t v, int n) { return (int32_t)((uint32_t)v << (n & 31)); }
static inline int32_t sar32(int32_t v, int n) { return v >> (n & 31); }
static inline uint32_t shr32u(uint32_t v, int n) { return v >> (n & 31); }
static inline int64_t shl64(int64_t v, int n) { return (int64_t)((uint64_t)v << (n & 63)); }
static inline int64_t sar64(int64_t v, int n) { return v >> (n & 63); }

/* checked array element access (IndexOutOfRangeException); the index
 * expression is evaluated exactly once (GNU statement expressions). */
#define B_AT(arr, len, i)                                                        \
    ({                                                                           \
        int64_t _bi = (int64_t)(i);                                              \
        if ((uint64_t)_bi >= (uint64_t)(int64_t)(len)) cs_throw(WVO_EXC_INDEX); \
        (arr)[_bi];                                                              \
    })
#define I_AT(arr, len, i)                                                        \
    (*({                                                                         \
        int64_t _ii = (int64_t)(i);                                              \
        if ((uint64_t)_ii >= (uint64_t)(int64_t)(len)) cs_throw(WVO_EXC_INDEX); \
        &(arr)[_ii];                                                             \
    }))

/* ------------------------------------------------------------------ */
/* State classes                                                       */
/* ------------------------------------------------------------------ */
typedef struct { /* Bitstream.cs:15-21 */
    int end, ptr;
    uint32_t sr;
    int file_bytes;
    int error, bc;
    uint8_t *buf;
    int buf_len;
    int buf_index;
    int valid; /* non-null reference */
} Bitstream;

typedef struct { /* decorr_pass.cs:24-26 */
    int16_t term, delta, weight_A, weight_B;
    int32_t samples_A[MAX_TERM];
    int32_t samples_B[MAX_TERM];
} decorr_pass;

typedef struct { /* entropy_data.cs:15-17 */
    int32_t slow_level;
    int32_t median[3];
    int32_t error_limit;
} entropy_data;

typedef struct { /* words_data.cs:23-29 */
    int64_t bitrate_delta[2];
    int64_t bitrate_acc[2];
    int64_t zeros_acc;
    int holding_one, holding_zero;
    entropy_data c[2];
} words_data;

typedef struct { /* WavpackHeader.cs:15-22 */
    uint32_t ckSize;
    int16_t version;
    int64_t total_samples, block_index;
    uint32_t block_samples, flags;
    int32_t crc;
    int error;
    int64_t stream_position;
    int64_t average_block_size;
} WavpackHeader;

typedef struct { /* WavpackStream.cs:15-19 */
    int32_t value, filter0, filter1, filter2, filter3, filter4, filter5, filter6, factor;
    int32_t bytei;
} DSDfilters;

typedef struct { /* WavpackStream.cs:21-35 */
    uint8_t *data;
    int data_len;
    int byteptr;
    uint8_t *probabilities;
    int probabilities_len;
    uint8_t *lookup_buffer;
    int lookup_len;
    int32_t *value_lookup;
    int value_lookup_len;
    uint8_t mode;
    int ready;
    int history_bins, p0, p1;
    uint16_t *summed_probabilities;
    int summed_len;
    uint32_t low, high, value;
    DSDfilters *filters; /* [2] */
    int32_t *ptable;     /* [256] */
} dsds;

typedef struct { /* WavpackStream.cs:47-84 */
    WavpackHeader wphdr;
    Bitstream wvbits, wvcbits, wvxbits;
    words_data w;
    int num_terms;
    int mute_error;
    int32_t crc, crc_x, crc_mvx;
    int64_t sample_index;
    int16_t int32_sent_bits, int32_zeros, int32_ones, int32_dups;
    int16_t float_flags, float_shift, float_max_exp, float_norm_exp;
    uint8_t int32_max_width;
    uint8_t float_min_shifted_zeros, float_max_shifted_ones;
    decorr_pass decorr_passes[MAX_NTERMS];
    dsds dsd;
} WavpackStream;

typedef struct { /* WavpackConfig.cs:15-18 */
    int bits_per_sample, bytes_per_sample;
    int num_channels, float_norm_exp;
    int64_t flags, sample_rate, channel_mask;
    uint8_t xmode;
} WavpackConfig;

typedef struct { /* in-memory System.IO.BinaryReader */
    const uint8_t *data;
    int64_t len, pos;
} Reader;

struct wvo_ctx { /* WavpackContext.cs:15-35 */
    WavpackConfig config;
    WavpackStream stream;
    uint8_t read_buffer[BITSTREAM_BUFFER_SIZE];
    const char *error_message;
    Reader infile;
    int64_t total_samples, crc_errors;
    int open_flags, norm_offset;
    int reduced_channels;
    int lossy_blocks;
    int five;
    int file_format;
    uint8_t *header;
    int header_len;
    uint8_t *trailer;
    int trailer_len;
    uint32_t dsd_multiplier;
    int exception;
    /* GC emulation: arrays released by their owner, freed at the next unpack_init */
    void **graveyard;
    int grave_n, grave_cap;
    char msgbuf[64];
};

typedef struct { /* WavpackMetadata.cs:15-23 */
    int byte_length;
    uint8_t *data;
    int data_len;
    int data_is_large; /* a private `new byte[]` not yet adopted by copy_data */
    uint8_t id;
    int hasdata;
    int error;
    int64_t bytecount;
} WavpackMetadata;

static void grave(wvo_ctx *ctx, void *p) {
    if (!p) return;
    if (ctx->grave_n == ctx->grave_cap) {
        ctx->grave_cap = ctx->grave_cap ? ctx->grave_cap * 2 : 16;
        ctx->graveyard = (void **)realloc(ctx->graveyard, sizeof(void *) * ctx->grave_cap);
    }
    ctx->graveyard[ctx->grave_n++] = p;
}
static void grave_flush(wvo_ctx *ctx) {
    for (int i = 0; i < ctx->grave_n; i++) free(ctx->graveyard[i]);
    ctx->grave_n = 0;
}

static void dsd_release(wvo_ctx *ctx, dsds *d) {
    grave(ctx, d->data);
    grave(ctx, d->probabilities);
    grave(ctx, d->lookup_buffer);
    grave(ctx, d->value_lookup);
    grave(ctx, d->summed_probabilities);
    grave(ctx, d->filters);
    grave(ctx, d->ptable);
    memset(d, 0, sizeof(*d));
}

/* Reader helpers: ReadByte throws EndOfStream (modelled as -1 to the caller
 * that catches it); BaseStream.Read returns a short count at EOF. */
static int rd_byte(Reader *r) {
    if (r->pos >= r->len) return -1;
    return r->data[r->pos++];
}
static int rd_read(Reader *r, uint8_t *dst, int n) {
    int64_t avail = r->len - r->pos;
    if (avail < 0) avail = 0;
    if (n > avail) n = (int)avail;
    if (n > 0) memcpy(dst, r->data + r->pos, (size_t)n);
    r->pos += n;
    return n;
}

/* ------------------------------------------------------------------ */
/* WordsUtils.cs tables (:33-66)                                       */
/* ------------------------------------------------------------------ */
static const int nbits_table[256] = {
    0, 1, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5,
    6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
    7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8,
    8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8,
    8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8,
    8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8};

static const int log2_table[256] = {
    0x00, 0x01, 0x03, 0x04, 0x06, 0x07, 0x09, 0x0a, 0x0b, 0x0d, 0x0e, 0x10, 0x11, 0x12, 0x14, 0x15,
    0x16, 0x18, 0x19, 0x1a, 0x1c, 0x1d, 0x1e, 0x20, 0x21, 0x22, 0x24, 0x25, 0x26, 0x28, 0x29, 0x2a,
    0x2c, 0x2d, 0x2e, 0x2f, 0x31, 0x32, 0x33, 0x34, 0x36, 0x37, 0x38, 0x39, 0x3b, 0x3c, 0x3d, 0x3e,
    0x3f, 0x41, 0x42, 0x43, 0x44, 0x45, 0x47, 0x48, 0x49, 0x4a, 0x4b, 0x4d, 0x4e, 0x4f, 0x50, 0x51,
    0x52, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x5c, 0x5d, 0x5e, 0x5f, 0x60, 0x61, 0x62, 0x63,
    0x64, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x6b, 0x6c, 0x6d, 0x6e, 0x6f, 0x70, 0x71, 0x72, 0x74, 0x75,
    0x76, 0x77, 0x78, 0x79, 0x7a, 0x7b, 0x7c, 0x7d, 0x7e, 0x7f, 0x80, 0x81, 0x82, 0x83, 0x84, 0x85,
    0x86, 0x87, 0x88, 0x89, 0x8a, 0x8b, 0x8c, 0x8d, 0x8e, 0x8f, 0x90, 0x91, 0x92, 0x93, 0x94, 0x95,
    0x96, 0x97, 0x98, 0x99, 0x9a, 0x9b, 0x9b, 0x9c, 0x9d, 0x9e, 0x9f, 0xa0, 0xa1, 0xa2, 0xa3, 0xa4,
    0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xa9, 0xaa, 0xab, 0xac, 0xad, 0xae, 0xaf, 0xb0, 0xb1, 0xb2, 0xb2,
    0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xb9, 0xba, 0xbb, 0xbc, 0xbd, 0xbe, 0xbf, 0xc0, 0xc0,
    0xc1, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xcb, 0xcb, 0xcc, 0xcd, 0xce,
    0xcf, 0xd0, 0xd0, 0xd1, 0xd2, 0xd3, 0xd4, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd8, 0xd9, 0xda, 0xdb,
    0xdc, 0xdc, 0xdd, 0xde, 0xdf, 0xe0, 0xe0, 0xe1, 0xe2, 0xe3, 0xe4, 0xe4, 0xe5, 0xe6, 0xe7, 0xe7,
    0xe8, 0xe9, 0xea, 0xea, 0xeb, 0xec, 0xed, 0xee, 0xee, 0xef, 0xf0, 0xf1, 0xf1, 0xf2, 0xf3, 0xf4,
    0xf4, 0xf5, 0xf6, 0xf7, 0xf7, 0xf8, 0xf9, 0xf9, 0xfa, 0xfb, 0xfc, 0xfc, 0xfd, 0xfe, 0xff, 0xff};

static const int exp2_table[256] = {
    0x00, 0x01, 0x01, 0x02, 0x03, 0x03, 0x04, 0x05, 0x06, 0x06, 0x07, 0x08, 0x08, 0x09, 0x0a, 0x0b,
    0x0b, 0x0c, 0x0d, 0x0e, 0x0e, 0x0f, 0x10, 0x10, 0x11, 0x12, 0x13, 0x13, 0x14, 0x15, 0x16, 0x16,
    0x17, 0x18, 0x19, 0x19, 0x1a, 0x1b, 0x1c, 0x1d, 0x1d, 0x1e, 0x1f, 0x20, 0x20, 0x21, 0x22, 0x23,
    0x24, 0x24, 0x25, 0x26, 0x27, 0x28, 0x28, 0x29, 0x2a, 0x2b, 0x2c, 0x2c, 0x2d, 0x2e, 0x2f, 0x30,
    0x30, 0x31, 0x32, 0x33, 0x34, 0x35, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x3a, 0x3b, 0x3c, 0x3d,
    0x3e, 0x3f, 0x40, 0x41, 0x41, 0x42, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x48, 0x49, 0x4a, 0x4b,
    0x4c, 0x4d, 0x4e, 0x4f, 0x50, 0x51, 0x51, 0x52, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a,
    0x5b, 0x5c, 0x5d, 0x5e, 0x5e, 0x5f, 0x60, 0x61, 0x62, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x6b, 0x6c, 0x6d, 0x6e, 0x6f, 0x70, 0x71, 0x72, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79,
    0x7a, 0x7b, 0x7c, 0x7d, 0x7e, 0x7f, 0x80, 0x81, 0x82, 0x83, 0x84, 0x85, 0x87, 0x88, 0x89, 0x8a,
    0x8b, 0x8c, 0x8d, 0x8e, 0x8f, 0x90, 0x91, 0x92, 0x93, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0x9b,
    0x9c, 0x9d, 0x9f, 0xa0, 0xa1, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa8, 0xa9, 0xaa, 0xab, 0xac, 0xad,
    0xaf, 0xb0, 0xb1, 0xb2, 0xb3, 0xb4, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xbc, 0xbd, 0xbe, 0xbf, 0xc0,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc8, 0xc9, 0xca, 0xcb, 0xcd, 0xce, 0xcf, 0xd0, 0xd2, 0xd3, 0xd4,
    0xd6, 0xd7, 0xd8, 0xd9, 0xdb, 0xdc, 0xdd, 0xde, 0xe0, 0xe1, 0xe2, 0xe4, 0xe5, 0xe6, 0xe8, 0xe9,
    0xea, 0xec, 0xed, 0xee, 0xf0, 0xf1, 0xf2, 0xf4, 0xf5, 0xf6, 0xf8, 0xf9, 0xfa, 0xfc, 0xfd, 0xff};

static const int ones_count_table[256] = {
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 5,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 6,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 5,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 7,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 5,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 6,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 5,
    0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 4, 0, 1, 0, 2, 0, 1, 0, 3, 0, 1, 0, 2, 0, 1, 0, 8};

static const int64_t sample_rates[15] = {6000,  8000,  9600,  11025, 12000, 16000, 22050, 24000,
                                         32000, 44100, 48000, 64000, 88200, 96000, 192000};

#define LIMIT_ONES 16
#define SLS 8
#define SLO (1 << (SLS - 1))
#define DIV0 128
#define DIV1 64
#define DIV2 32

/* ------------------------------------------------------------------ */
/* BitsUtils.cs                                                        */
/* ------------------------------------------------------------------ */
static void bs_read(Bitstream *bs) /* BitsUtils.cs:95-146 (file_bytes is always 0 here) */
{
    /* UnpackUtils.cs:82,103,130 all pass file_bytes = 0, so only the
     * error branch (:132-140) is reachable: fill the whole array with 0xFF. */
    bs->error = 1;
    memset(bs->buf, 0xFF, (size_t)bs->buf_len);
    bs->ptr = 0;
    bs->buf_index = 0;
}

static int getbit(Bitstream *bs) /* BitsUtils.cs:15-35 */
{
    if (bs->bc > 0)
        bs->bc--;
    else {
        bs->ptr++;
        bs->buf_index++;
        bs->bc = 7;
        if (bs->ptr == bs->end) bs_read(bs);
        bs->sr = B_AT(bs->buf, bs->buf_len, bs->buf_index);
    }
    int result = (bs->sr & 1) > 0;
    bs->sr >>= 1;
    return result;
}

static int64_t getbits(int nbits, Bitstream *bs) /* BitsUtils.cs:37-68 */
{
    int64_t retval;
    while (nbits > bs->bc) {
        bs->ptr++;
        bs->buf_index++;
        if (bs->ptr == bs->end) bs_read(bs);
        bs->sr |= (uint32_t)shl32((int32_t)B_AT(bs->buf, bs->buf_len, bs->buf_index), bs->bc);
        bs->bc += 8;
    }
    retval = (int64_t)bs->sr;
    if (bs->bc > 32) {
        bs->bc -= nbits;
        bs->sr = (uint32_t)sar32((int32_t)B_AT(bs->buf, bs->buf_len, bs->buf_index), 8 - bs->bc);
    } else {
        bs->bc -= nbits;
        bs->sr = shr32u(bs->sr, nbits);
    }
    return retval;
}

static Bitstream bs_open_read(uint8_t *stream, int stream_len, int buffer_start, int buffer_end) /* BitsUtils.cs:70-93, passed=0 */
{
    Bitstream bs;
    memset(&bs, 0, sizeof(bs));
    bs.buf = stream;
    bs.buf_len = stream_len;
    bs.buf_index = buffer_start;
    bs.end = buffer_end;
    bs.sr = 0;
    bs.bc = 0;
    bs.buf_index--;
    bs.ptr = -1;
    bs.valid = 1;
    return bs;
}

/* ------------------------------------------------------------------ */
/* WordsUtils.cs                                                       */
/* ------------------------------------------------------------------ */
static int count_bits(int64_t av) /* WordsUtils.cs:513-537 */
{
    if (av < 256) return B_AT(nbits_table, 256, av);
    if (av < 65536) return B_AT(nbits_table, 256, av >> 8) + 8;
    if (av < 16777216) return B_AT(nbits_table, 256, av >> 16) + 16;
    return B_AT(nbits_table, 256, av >> 24) + 24;
}

static int exp2s(int log) /* WordsUtils.cs:633-646 */
{
    int64_t value;
    if (log == INT32_MIN) cs_throw(WVO_EXC_STACK); /* C#: -exp2s(-int.MinValue) recurses forever */
    if (log < 0) return -exp2s(-log);
    value = exp2_table[log & 0xff] | 0x100;
    if ((log >>= 8) <= 9)
        return (int)sar64(value, 9 - log);
    else
        return (int)shl64(value, log - 9);
}

static int mylog2(int64_t avalue) /* WordsUtils.cs:588-608 */
{
    int dbits;
    if ((avalue += (avalue >> 9)) < (1 << 8)) {
        dbits = B_AT(nbits_table, 256, (int32_t)avalue);
        return (dbits << 8) + log2_table[(int)shl64(avalue, 9 - dbits) & 0xff];
    } else {
        if (avalue < (1LL << 16))
            dbits = B_AT(nbits_table, 256, (int32_t)(avalue >> 8)) + 8;
        else if (avalue < (1LL << 24))
            dbits = B_AT(nbits_table, 256, (int32_t)(avalue >> 16)) + 16;
        else
            dbits = B_AT(nbits_table, 256, (int32_t)(avalue >> 24)) + 24;
        return (dbits << 8) + log2_table[(int)sar64(avalue, dbits - 9) & 0xff];
    }
}

static int restore_weight(int8_t weight) /* WordsUtils.cs:653-661 */
{
    int result;
    if ((result = weight * 8) > 0) result += (result + 64) >> 7;
    return result;
}

static int64_t read_code(Bitstream *bs, int64_t maxcode) /* WordsUtils.cs:546-570 */
{
    int bitcount = count_bits(maxcode);
    int64_t extras = (int64_t)shl32(1, bitcount) - maxcode - 1;
    int64_t code;
    if (bitcount == 0) return 0;
    code = getbits(bitcount - 1, bs);
    code &= (int64_t)(shl32(1, bitcount - 1) - 1);
    if (code >= extras) {
        code = (code << 1) - extras;
        if (getbit(bs)) ++code;
    }
    return code;
}

static void update_error_limit(words_data *w, int64_t flags) /* WordsUtils.cs:195-261 */
{
    int bitrate_0 = (int)((w->bitrate_acc[0] += w->bitrate_delta[0]) >> 16);
    if ((flags & MONO_DATA) != 0) {
        if ((flags & HYBRID_BITRATE) != 0) {
            int slow_log_0 = (int)((w->c[0].slow_level + SLO) >> SLS);
            if (slow_log_0 - bitrate_0 > -0x100)
                w->c[0].error_limit = exp2s(slow_log_0 - bitrate_0 + 0x100);
            else
                w->c[0].error_limit = 0;
        } else
            w->c[0].error_limit = exp2s(bitrate_0);
    } else {
        int bitrate_1 = (int)((w->bitrate_acc[1] += w->bitrate_delta[1]) >> 16);
        if ((flags & HYBRID_BITRATE) != 0) {
            int slow_log_0 = (int)((w->c[0].slow_level + SLO) >> SLS);
            int slow_log_1 = (int)((w->c[1].slow_level + SLO) >> SLS);
            if ((flags & HYBRID_BALANCE) != 0) {
                int balance = (slow_log_1 - slow_log_0 + bitrate_1 + 1) >> 1;
                if (balance > bitrate_0) {
                    bitrate_1 = bitrate_0 * 2;
                    bitrate_0 = 0;
                } else if (-balance > bitrate_0) {
                    bitrate_0 = bitrate_0 * 2;
                    bitrate_1 = 0;
                } else {
                    bitrate_1 = bitrate_0 + balance;
                    bitrate_0 = bitrate_0 - balance;
                }
            }
            if (slow_log_0 - bitrate_0 > -0x100)
                w->c[0].error_limit = exp2s(slow_log_0 - bitrate_0 + 0x100);
            else
                w->c[0].error_limit = 0;
            if (slow_log_1 - bitrate_1 > -0x100)
                w->c[1].error_limit = exp2s(slow_log_1 - bitrate_1 + 0x100);
            else
                w->c[1].error_limit = 0;
        } else {
            w->c[0].error_limit = exp2s(bitrate_0);
            w->c[1].error_limit = exp2s(bitrate_1);
        }
    }
}

/* WordsUtils.cs:272-511 */
static int get_words(int64_t nsamples, int64_t flags, words_data *w, Bitstream *bs, int32_t *buffer,
                     int64_t buffer_len, int bufferStartPos)
{
    entropy_data *c = w->c;
    int csamples;
    int buffer_counter = bufferStartPos;
    int entidx = 1;

    if ((flags & MONO_DATA) == 0)
        nsamples *= 2;
    else
        entidx = 0;

    for (csamples = 0; csamples < nsamples; ++csamples) {
        int ones_count;
        int64_t low, high, mid;

        if ((flags & MONO_DATA) == 0) entidx = (entidx == 1) ? 0 : 1;

        if ((w->c[0].median[0] & ~1) == 0 && !w->holding_zero && !w->holding_one &&
            (w->c[1].median[0] & ~1) == 0) {
            int64_t mask;
            int cbits;

            if (w->zeros_acc > 0) {
                if (--w->zeros_acc > 0) {
                    c[entidx].slow_level -= (c[entidx].slow_level + SLO) >> SLS;
                    I_AT(buffer, buffer_len, buffer_counter) = 0;
                    buffer_counter++;
                    continue;
                }
            } else {
                for (cbits = 0; cbits < 33 && getbit(bs); ++cbits)
                    ;
                if (cbits == 33) break;
                if (cbits < 2)
                    w->zeros_acc = cbits;
                else {
                    for (mask = 1, w->zeros_acc = 0; --cbits > 0; mask <<= 1)
                        if (getbit(bs)) w->zeros_acc |= mask;
                    w->zeros_acc |= mask;
                }
                if (w->zeros_acc > 0) {
                    c[entidx].slow_level -= ((c[entidx].slow_level + SLO) >> SLS);
                    w->c[0].median[0] = 0;
                    w->c[0].median[1] = 0;
                    w->c[0].median[2] = 0;
                    w->c[1].median[0] = 0;
                    w->c[1].median[1] = 0;
                    w->c[1].median[2] = 0;
                    I_AT(buffer, buffer_len, buffer_counter) = 0;
                    buffer_counter++;
                    continue;
                }
            }
        }

        if (w->holding_zero) {
            w->holding_zero = 0;
            ones_count = 0;
        } else {
            if (bs->bc < 8) {
                bs->ptr++;
                bs->buf_index++;
                if (bs->ptr == bs->end) bs_read(bs);
                bs->sr |= (uint32_t)shl32((int32_t)B_AT(bs->buf, bs->buf_len, bs->buf_index), bs->bc);
                bs->bc += 8;
            }
            uint8_t next8 = (uint8_t)bs->sr;
            if (next8 == 0xff) {
                bs->bc -= 8;
                bs->sr >>= 8;
                for (ones_count = 8; ones_count < (LIMIT_ONES + 1) && getbit(bs); ++ones_count)
                    ;
                if (ones_count == (LIMIT_ONES + 1)) break;
                if (ones_count == LIMIT_ONES) {
                    int mask;
                    int cbits;
                    for (cbits = 0; cbits < 33 && getbit(bs); ++cbits)
                        ;
                    if (cbits == 33) break;
                    if (cbits < 2)
                        ones_count = cbits;
                    else {
                        for (mask = 1, ones_count = 0; --cbits > 0; mask = shl32(mask, 1))
                            if (getbit(bs)) ones_count |= mask;
                        ones_count |= mask;
                    }
                    ones_count += LIMIT_ONES;
                }
            } else {
                bs->bc -= (ones_count = ones_count_table[next8]) + 1;
                bs->sr = shr32u(bs->sr, ones_count + 1);
            }
            if (w->holding_one) {
                w->holding_one = (ones_count & 1) > 0;
                ones_count = (ones_count >> 1) + 1;
            } else {
                w->holding_one = (ones_count & 1) > 0;
                ones_count >>= 1;
            }
            w->holding_zero = !w->holding_one;
        }

        if ((flags & HYBRID_FLAG) > 0 && ((flags & MONO_DATA) > 0 || (csamples & 1) == 0))
            update_error_limit(w, flags);

        if (ones_count == 0) {
            low = 0;
            high = (int64_t)(((c[entidx].median[0]) >> 4) + 1) - 1;
            c[entidx].median[0] -= (((c[entidx].median[0] + (DIV0 - 2)) >> 7) * 2);
        } else {
            low = (((c[entidx].median[0]) >> 4) + 1);
            c[entidx].median[0] += ((c[entidx].median[0] + DIV0) >> 7) * 5;
            if (ones_count == 1) {
                high = low + (((c[entidx].median[1]) >> 4) + 1) - 1;
                c[entidx].median[1] -= ((c[entidx].median[1] + (DIV1 - 2)) >> 6) * 2;
            } else {
                low += (((c[entidx].median[1]) >> 4) + 1);
                c[entidx].median[1] += ((c[entidx].median[1] + DIV1) >> 6) * 5;
                if (ones_count == 2) {
                    high = low + (((c[entidx].median[2]) >> 4) + 1) - 1;
                    c[entidx].median[2] -= ((c[entidx].median[2] + (DIV2 - 2)) >> 5) * 2;
                } else {
                    low += (int64_t)(int32_t)((ones_count - 2) * (((c[entidx].median[2]) >> 4) + 1));
                    high = low + (((c[entidx].median[2]) >> 4) + 1) - 1;
                    c[entidx].median[2] += ((c[entidx].median[2] + DIV2) >> 5) * 5;
                }
            }
        }

        mid = (high + low + 1) >> 1;

        if (c[entidx].error_limit == 0) {
            mid = read_code(bs, high - low);
            mid = mid + low;
        } else {
            /* The C# loop (WordsUtils.cs:486-492) never ends for some negative
             * error limits: from any start high-low settles into {-2,-1,0} within
             * ~70 steps; there -1 is a fixed point, 0 waits for a 0 bit (none past
             * the payload's end) and nothing exits below -2.  Report it as the
             * exception it stands for instead of looping; 2^24 steps exceed every
             * bit of a < 1 MiB block, so no terminating loop is cut short. */
            int64_t steps = 0;
            while (high - low > c[entidx].error_limit) {
                if (++steps > 72) {
                    int64_t d = high - low;
                    if ((d >= -2 && d <= 0 && (c[entidx].error_limit <= -3 || d == -1)) || steps > (1 << 24))
                        cs_throw(WVO_EXC_HANG);
                }
                if (getbit(bs))
                    mid = (high + (low = mid) + 1) >> 1;
                else
                    mid = ((high = mid - 1) + low + 1) >> 1;
            }
        }

        if (getbit(bs))
            I_AT(buffer, buffer_len, buffer_counter) = (int32_t)~mid;
        else
            I_AT(buffer, buffer_len, buffer_counter) = (int32_t)mid;
        buffer_counter++;

        if ((flags & HYBRID_BITRATE) > 0)
            c[entidx].slow_level = c[entidx].slow_level - ((c[entidx].slow_level + SLO) >> SLS) + mylog2(mid);
    }

    if ((flags & MONO_DATA) != 0)
        return csamples;
    else
        return csamples / 2;
}

static int read_entropy_vars(WavpackStream *wps, WavpackMetadata *wpmd) /* WordsUtils.cs:75-116 */
{
    const uint8_t *byteptr = wpmd->data;
    int b_array[12];
    int i;
    words_data w;
    memset(&w, 0, sizeof(w));

    for (i = 0; i < 6; i++) b_array[i] = B_AT(byteptr, wpmd->data_len, i);
    w.holding_one = 0;
    w.holding_zero = 0;
    if (wpmd->byte_length != 12) {
        if ((wps->wphdr.flags & MONO_DATA) == 0) return 0;
    }
    w.c[0].median[0] = exp2s(b_array[0] + (b_array[1] << 8));
    w.c[0].median[1] = exp2s(b_array[2] + (b_array[3] << 8));
    w.c[0].median[2] = exp2s(b_array[4] + (b_array[5] << 8));
    if ((wps->wphdr.flags & MONO_DATA) == 0) {
        for (i = 6; i < 12; i++) b_array[i] = B_AT(byteptr, wpmd->data_len, i);
        w.c[1].median[0] = exp2s(b_array[6] + (b_array[7] << 8));
        w.c[1].median[1] = exp2s(b_array[8] + (b_array[9] << 8));
        w.c[1].median[2] = exp2s(b_array[10] + (b_array[11] << 8));
    }
    wps->w = w;
    return 1;
}

static int read_hybrid_profile(WavpackStream *wps, WavpackMetadata *wpmd) /* WordsUtils.cs:124-187 */
{
    const uint8_t *byteptr = wpmd->data;
    int n = wpmd->data_len;
    int bytecnt = wpmd->byte_length;
    int bc = 0;
    int u0, u1;

    if ((wps->wphdr.flags & HYBRID_BITRATE) != 0) {
        u0 = B_AT(byteptr, n, bc);
        u1 = B_AT(byteptr, n, bc + 1);
        wps->w.c[0].slow_level = exp2s(u0 + (u1 << 8));
        bc += 2;
        if ((wps->wphdr.flags & MONO_DATA) == 0) {
            u0 = B_AT(byteptr, n, bc);
            u1 = B_AT(byteptr, n, bc + 1);
            wps->w.c[1].slow_level = exp2s(u0 + (u1 << 8));
            bc += 2;
        }
    }
    u0 = B_AT(byteptr, n, bc);
    u1 = B_AT(byteptr, n, bc + 1);
    wps->w.bitrate_acc[0] = (int64_t)shl32(u0 + (u1 << 8), 16);
    bc += 2;
    if ((wps->wphdr.flags & MONO_DATA) == 0) {
        u0 = B_AT(byteptr, n, bc);
        u1 = B_AT(byteptr, n, bc + 1);
        wps->w.bitrate_acc[1] = (int64_t)shl32(u0 + (u1 << 8), 16);
        bc += 2;
    }
    if (bc < bytecnt) {
        u0 = B_AT(byteptr, n, bc);
        u1 = B_AT(byteptr, n, bc + 1);
        wps->w.bitrate_delta[0] = exp2s((int16_t)(u0 + (u1 << 8)));
        bc += 2;
        if ((wps->wphdr.flags & MONO_DATA) == 0) {
            u0 = B_AT(byteptr, n, bc);
            u1 = B_AT(byteptr, n, bc + 1);
            wps->w.bitrate_delta[1] = exp2s((int16_t)(u0 + (u1 << 8)));
            bc += 2;
        }
        if (bc < bytecnt) return 0;
    } else
        wps->w.bitrate_delta[0] = wps->w.bitrate_delta[1] = 0;
    return 1;
}

/* ------------------------------------------------------------------ */
/* FloatUtils.cs                                                       */
/* ------------------------------------------------------------------ */
static int read_float_info(WavpackStream *wps, WavpackMetadata *wpmd) /* FloatUtils.cs:15-30 */
{
    if (wpmd->byte_length != 4) return 0;
    wps->float_flags = B_AT(wpmd->data, wpmd->data_len, 0);
    wps->float_shift = B_AT(wpmd->data, wpmd->data_len, 1);
    wps->float_max_exp = B_AT(wpmd->data, wpmd->data_len, 2);
    wps->float_norm_exp = B_AT(wpmd->data, wpmd->data_len, 3);
    return 1;
}

static void float_values(WavpackStream *wps, int32_t *values, int64_t vlen, int64_t num_values,
                         int bufferStartPos) /* FloatUtils.cs:32-56 */
{
    int shift = wps->float_max_exp - wps->float_norm_exp + wps->float_shift;
    int vc = bufferStartPos;
    if (shift > 32)
        shift = 32;
    else if (shift < -32)
        shift = -32;
    while (num_values-- > 0) {
        int32_t *v = &I_AT(values, vlen, vc);
        if (shift > 0)
            *v = shl32(*v, shift);
        else if (shift < 0)
            *v = sar32(*v, -shift);
        if (*v > 8388607)
            *v = 8388607;
        else if (*v < -8388608)
            *v = -8388608;
        vc++;
    }
}

/* ------------------------------------------------------------------ */
/* WavpackMetadata.copy_data (WavpackMetadata.cs:25-36)                */
/* Returns the adopted array (ownership passes to the caller) or NULL. */
/* ------------------------------------------------------------------ */
static uint8_t *copy_data(WavpackMetadata *m, int *out_len)
{
    if (!m->hasdata || m->byte_length <= 0) return NULL;
    if (m->data_len != BITSTREAM_BUFFER_SIZE) {
        m->data_is_large = 0; /* adopted */
        *out_len = m->data_len;
        return m->data;
    }
    uint8_t *nd = (uint8_t *)malloc((size_t)m->byte_length);
    memcpy(nd, m->data, (size_t)m->byte_length);
    m->data = nd;
    m->data_len = m->byte_length;
    m->data_is_large = 0;
    *out_len = m->byte_length;
    return nd;
}

/* ------------------------------------------------------------------ */
/* UnpackUtils.cs metadata readers                                     */
/* ------------------------------------------------------------------ */
static void replace_bits(wvo_ctx *ctx, Bitstream *slot, Bitstream nb)
{
    if (slot->valid) grave(ctx, slot->buf);
    *slot = nb;
}

static int init_wv_bitstream(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:74-90 */
{
    int len;
    uint8_t *d = copy_data(wpmd, &len);
    if (!d) return 0;
    replace_bits(wpc, &wpc->stream.wvbits, bs_open_read(d, len, 0, wpmd->byte_length));
    return 1;
}

static int init_wvc_bitstream(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:96-106 */
{
    int len;
    if ((wpmd->byte_length & 1) > 0) return 0;
    uint8_t *d = copy_data(wpmd, &len);
    if (!d) return 0;
    replace_bits(wpc, &wpc->stream.wvcbits, bs_open_read(d, len, 0, wpmd->byte_length));
    return 1;
}

static int init_wvx_bitstream(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:115-147 */
{
    WavpackStream *wps = &wpc->stream;
    int counter = 0, len;
    uint8_t *d;
    if (wpmd->byte_length <= 4 || (wpmd->byte_length & 1) > 0) return 0;
    d = copy_data(wpmd, &len);
    if (!d) return 0;
    int cp = B_AT(d, len, counter);
    counter++;
    wps->crc_mvx = cp;
    wps->crc_mvx |= B_AT(d, len, counter) << 8;
    counter++;
    wps->crc_mvx |= B_AT(d, len, counter) << 16;
    counter++;
    wps->crc_mvx |= shl32(B_AT(d, len, counter), 24);
    counter++;
    replace_bits(wpc, &wps->wvxbits, bs_open_read(d, len, counter, wpmd->byte_length));
    if (wpmd->id == ID_WVX_NEW_BITSTREAM) {
        if ((wps->wphdr.flags & FLOAT_DATA) > 0) {
            wps->float_min_shifted_zeros = (uint8_t)(getbits(5, &wps->wvxbits) & 0x1f);
            wps->float_max_shifted_ones = (uint8_t)(getbits(5, &wps->wvxbits) & 0x1f);
        } else
            wps->int32_max_width = (uint8_t)(getbits(5, &wps->wvxbits) & 0x1f);
    }
    return 1;
}

static int read_decorr_terms(WavpackStream *wps, WavpackMetadata *wpmd) /* UnpackUtils.cs:156-187 */
{
    int termcnt = wpmd->byte_length;
    decorr_pass tmp[MAX_NTERMS];
    int counter = 0, dcounter;
    if (termcnt > MAX_NTERMS) return 0;
    memset(tmp, 0, sizeof(tmp)); /* `new WavpackStream()` -> fresh passes */
    for (dcounter = termcnt - 1; dcounter >= 0; dcounter--) {
        int b = B_AT(wpmd->data, wpmd->data_len, counter);
        tmp[dcounter].term = (int16_t)((b & 0x1f) - 5);
        tmp[dcounter].delta = (int16_t)((b >> 5) & 0x7);
        counter++;
        if (tmp[dcounter].term < -3 || (tmp[dcounter].term > MAX_TERM && tmp[dcounter].term < 17) ||
            tmp[dcounter].term > 18)
            return 0;
    }
    memcpy(wps->decorr_passes, tmp, sizeof(tmp));
    wps->num_terms = termcnt;
    return 1;
}

static int read_decorr_weights(WavpackStream *wps, WavpackMetadata *wpmd) /* UnpackUtils.cs:196-239 */
{
    int termcnt = wpmd->byte_length, tcount;
    int counter = 0, dpp_idx, myiterator;
    int16_t dw_A = 0, dw_B = 0;
    if ((wps->wphdr.flags & MONO_DATA) == 0) termcnt /= 2;
    if (termcnt > wps->num_terms) return 0;
    for (tcount = wps->num_terms; tcount > 0; tcount--) dw_A = dw_B = 0;
    myiterator = wps->num_terms;
    while (termcnt > 0) {
        dpp_idx = myiterator - 1;
        dw_A = (int16_t)restore_weight((int8_t)B_AT(wpmd->data, wpmd->data_len, counter));
        I_AT(wps->decorr_passes, MAX_NTERMS, dpp_idx).weight_A = dw_A;
        counter++;
        if ((wps->wphdr.flags & MONO_DATA) == 0) {
            dw_B = (int16_t)restore_weight((int8_t)B_AT(wpmd->data, wpmd->data_len, counter));
            counter++;
        }
        I_AT(wps->decorr_passes, MAX_NTERMS, dpp_idx).weight_B = dw_B;
        myiterator--;
        termcnt--;
    }
    return 1;
}

static int read_decorr_samples(WavpackStream *wps, WavpackMetadata *wpmd) /* UnpackUtils.cs:250-360 */
{
    const uint8_t *bp = wpmd->data;
    int n = wpmd->data_len;
    decorr_pass dpp;
    int tcount, counter = 0, dpp_index = 0, sc;
    int u0, u1, u2, u3;
    memset(&dpp, 0, sizeof(dpp));

    for (tcount = wps->num_terms; tcount > 0; tcount--) {
        dpp.term = I_AT(wps->decorr_passes, MAX_NTERMS, dpp_index).term;
        for (int ic = 0; ic < MAX_TERM; ic++) {
            dpp.samples_A[ic] = 0;
            dpp.samples_B[ic] = 0;
            wps->decorr_passes[dpp_index].samples_A[ic] = 0;
            wps->decorr_passes[dpp_index].samples_B[ic] = 0;
        }
        dpp_index++;
    }
    if (wps->wphdr.version == 0x402 && (wps->wphdr.flags & HYBRID_FLAG) > 0) {
        counter += 2;
        if ((wps->wphdr.flags & MONO_DATA) == 0) counter += 2;
    }
    dpp_index--;
    while (counter < wpmd->byte_length) {
        if (dpp.term > MAX_TERM) {
            u0 = B_AT(bp, n, counter); u1 = B_AT(bp, n, counter + 1);
            u2 = B_AT(bp, n, counter + 2); u3 = B_AT(bp, n, counter + 3);
            dpp.samples_A[0] = exp2s((int16_t)(u0 + (u1 << 8)));
            dpp.samples_A[1] = exp2s((int16_t)(u2 + (u3 << 8)));
            counter += 4;
            if ((wps->wphdr.flags & MONO_DATA) == 0) {
                u0 = B_AT(bp, n, counter); u1 = B_AT(bp, n, counter + 1);
                u2 = B_AT(bp, n, counter + 2); u3 = B_AT(bp, n, counter + 3);
                dpp.samples_B[0] = exp2s((int16_t)(u0 + (u1 << 8)));
                dpp.samples_B[1] = exp2s((int16_t)(u2 + (u3 << 8)));
                counter += 4;
            }
        } else if (dpp.term < 0) {
            u0 = B_AT(bp, n, counter); u1 = B_AT(bp, n, counter + 1);
            u2 = B_AT(bp, n, counter + 2); u3 = B_AT(bp, n, counter + 3);
            dpp.samples_A[0] = exp2s((int16_t)(u0 + (u1 << 8)));
            dpp.samples_B[0] = exp2s((int16_t)(u2 + (u3 << 8)));
            counter += 4;
        } else {
            int m = 0, cnt = dpp.term;
            while (cnt > 0) {
                u0 = B_AT(bp, n, counter); u1 = B_AT(bp, n, counter + 1);
                dpp.samples_A[m] = exp2s((int16_t)(u0 + (u1 << 8)));
                counter += 2;
                if ((wps->wphdr.flags & MONO_DATA) == 0) {
                    u0 = B_AT(bp, n, counter); u1 = B_AT(bp, n, counter + 1);
                    dpp.samples_B[m] = exp2s((int16_t)(u0 + (u1 << 8)));
                    counter += 2;
                }
                m++;
                cnt--;
            }
        }
        for (sc = 0; sc < MAX_TERM; sc++) {
            I_AT(wps->decorr_passes, MAX_NTERMS, dpp_index).samples_A[sc] = dpp.samples_A[sc];
            wps->decorr_passes[dpp_index].samples_B[sc] = dpp.samples_B[sc];
        }
        dpp_index--;
    }
    return 1;
}

static int read_int32_info(WavpackStream *wps, WavpackMetadata *wpmd) /* UnpackUtils.cs:367-382 */
{
    if (wpmd->byte_length != 4) return 0;
    wps->int32_sent_bits = B_AT(wpmd->data, wpmd->data_len, 0);
    wps->int32_zeros = B_AT(wpmd->data, wpmd->data_len, 1);
    wps->int32_ones = B_AT(wpmd->data, wpmd->data_len, 2);
    wps->int32_dups = B_AT(wpmd->data, wpmd->data_len, 3);
    return 1;
}

static int read_channel_info(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:389-410 */
{
    int bytecnt = wpmd->byte_length, shift = 0, counter = 0;
    int64_t mask = 0;
    if (bytecnt == 0 || bytecnt > 5) return 0;
    wpc->config.num_channels = B_AT(wpmd->data, wpmd->data_len, counter);
    counter++;
    while (bytecnt >= 0) {
        mask |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, counter), shift);
        counter++;
        shift += 8;
        bytecnt--;
    }
    wpc->config.channel_mask = mask;
    return 1;
}

static int read_new_config_info(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:415-427 */
{
    wpc->five = 1;
    if (wpmd->byte_length >= 1) wpc->file_format = B_AT(wpmd->data, wpmd->data_len, 0);
    return 1;
}

static int read_config_info(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:432-455 */
{
    int bytecnt = wpmd->byte_length, counter = 0;
    if (bytecnt >= 3) {
        wpc->config.flags &= 0xff;
        wpc->config.flags |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, counter), 8);
        counter++;
        wpc->config.flags |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, counter), 16);
        counter++;
        wpc->config.flags |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, counter), 24);
        counter++;
    }
    if (bytecnt >= 4 && (wpc->config.flags & CONFIG_EXTRA_MODE) > 0) {
        wpc->config.xmode = B_AT(wpmd->data, wpmd->data_len, counter);
        counter++;
        bytecnt--;
    }
    if (bytecnt >= 5) wpc->five = 1;
    return 1;
}

static int read_sample_rate(wvo_ctx *wpc, WavpackMetadata *wpmd) /* UnpackUtils.cs:459-473 */
{
    if (wpmd->byte_length == 3) {
        wpc->config.sample_rate = B_AT(wpmd->data, wpmd->data_len, 0);
        wpc->config.sample_rate |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, 1), 8);
        wpc->config.sample_rate |= (int64_t)shl32(B_AT(wpmd->data, wpmd->data_len, 2), 16);
    }
    return 1;
}

static int read_header_md(wvo_ctx *wpc, WavpackMetadata *wpmd, int trailer) /* UnpackUtils.cs:475-491 */
{
    int n = wpmd->byte_length;
    if (n < 0) cs_throw(WVO_EXC_INDEX); /* new byte[-1] -> OverflowException */
    if (n > wpmd->data_len) cs_throw(WVO_EXC_INDEX);
    uint8_t *b = (uint8_t *)malloc((size_t)(n ? n : 1));
    memcpy(b, wpmd->data, (size_t)n);
    if (trailer) {
        free(wpc->trailer);
        wpc->trailer = b;
        wpc->trailer_len = n;
    } else {
        free(wpc->header);
        wpc->header = b;
        wpc->header_len = n;
    }
    return 1;
}

/* ------------------------------------------------------------------ */
/* DsdUtils.cs                                                         */
/* ------------------------------------------------------------------ */
#define MAX_HISTORY_BITS 5
#define MAX_BYTES_PER_BIN 1280
#define MAX_DSD_BITS_VALUE 256
#define PTABLE_BITS 8
#define PTABLE_BINS (1 << PTABLE_BITS)
#define PTABLE_MASK (PTABLE_BINS - 1)
#define UP 0x010000FE
#define DOWN 0x00010000
#define DECAY 8
#define PRECISION 20
#define VALUE_ONE (1 << PRECISION)
#define PRECISION_USE 12
#define RATE_S 20

static int init_dsd_block_fast(WavpackStream *wps) /* DsdUtils.cs:149-242 */
{
    dsds *d = &wps->dsd;
    uint8_t max_probability;
    int total_summed_probabilities = 0, bi, i;
    if (d->byteptr == d->data_len) return 0;
    uint8_t history_bits = B_AT(d->data, d->data_len, d->byteptr);
    d->byteptr++;
    if (d->byteptr == d->data_len || history_bits > MAX_HISTORY_BITS) return 0;
    d->history_bins = 1 << history_bits;
    d->lookup_len = d->history_bins * MAX_BYTES_PER_BIN;
    d->lookup_buffer = (uint8_t *)calloc((size_t)d->lookup_len, 1);
    d->value_lookup_len = d->history_bins;
    d->value_lookup = (int32_t *)calloc((size_t)d->history_bins, sizeof(int32_t));
    d->summed_len = MAX_DSD_BITS_VALUE * d->history_bins;
    d->summed_probabilities = (uint16_t *)calloc((size_t)d->summed_len, sizeof(uint16_t));
    d->probabilities_len = MAX_DSD_BITS_VALUE * d->history_bins;
    d->probabilities = (uint8_t *)calloc((size_t)d->probabilities_len, 1);

    max_probability = B_AT(d->data, d->data_len, d->byteptr);
    d->byteptr++;
    if (max_probability < 0xFF) {
        int outptr = 0, outend = d->probabilities_len;
        while (outptr < outend && d->byteptr < d->data_len) {
            uint8_t code = d->data[d->byteptr++];
            if (code > max_probability) {
                int zcount = code - max_probability;
                while (outptr < outend && zcount-- > 0) d->probabilities[outptr++] = 0;
            } else if (code != 0)
                d->probabilities[outptr++] = code;
            else
                break;
        }
        if (outptr < outend || (d->byteptr < d->data_len && d->data[d->byteptr++] > 0)) return 0;
    } else if (d->data_len - d->byteptr > d->probabilities_len) {
        memcpy(d->probabilities, d->data + d->byteptr, (size_t)d->probabilities_len);
        d->byteptr += d->probabilities_len;
    } else
        return 0;

    int lb_ptr = 0;
    for (bi = 0; bi < d->history_bins; ++bi) {
        uint16_t sum_values;
        int bi_index = bi * MAX_DSD_BITS_VALUE;
        for (sum_values = 0, i = 0; i < MAX_DSD_BITS_VALUE; ++i)
            d->summed_probabilities[bi_index + i] = sum_values = (uint16_t)(sum_values + d->probabilities[bi_index + i]);
        if (sum_values != 0) {
            if ((total_summed_probabilities += sum_values) > d->history_bins * MAX_BYTES_PER_BIN) return 0;
            d->value_lookup[bi] = lb_ptr;
            for (i = 0; i < MAX_DSD_BITS_VALUE; i++) {
                int c = d->probabilities[bi_index + i];
                while (c-- > 0) {
                    I_AT(d->lookup_buffer, d->lookup_len, lb_ptr) = (uint8_t)i;
                    lb_ptr++;
                }
            }
        }
    }
    if (d->data_len - d->byteptr < 4 || total_summed_probabilities > d->history_bins * MAX_BYTES_PER_BIN) return 0;
    for (i = 4; i > 0; i--) {
        d->value = (d->value << 8) | d->data[d->byteptr];
        d->byteptr++;
    }
    d->p0 = d->p1 = 0;
    d->low = 0;
    d->high = 0xFFFFFFFFu;
    d->ready = 1;
    return 1;
}

static int64_t decode_fast(WavpackStream *wps, int32_t *output, int64_t olen, int64_t sample_count,
                           int bufferStartPos) /* DsdUtils.cs:244-304 */
{
    dsds *d = &wps->dsd;
    int64_t total_samples = sample_count;
    if ((wps->wphdr.flags & MONO_DATA) == 0) total_samples *= 2;
    while (total_samples-- > 0) {
        uint32_t mult, index, i;
        int code;
        int p0_index = d->p0 * MAX_DSD_BITS_VALUE;
        uint16_t tot = I_AT(d->summed_probabilities, d->summed_len, p0_index + 255);
        if (tot == 0) return 0;
        mult = (d->high - d->low) / tot;
        if (mult == 0) {
            if (d->data_len - d->byteptr >= 4)
                for (i = 4; i > 0; i--) {
                    d->value = (d->value << 8) | d->data[d->byteptr];
                    d->byteptr++;
                }
            d->low = 0;
            d->high = 0xFFFFFFFFu;
            mult = d->high / tot;
            if (mult == 0) return 0;
        }
        index = (d->value - d->low) / mult;
        if (index >= tot) return 0;
        code = I_AT(d->lookup_buffer, d->lookup_len, (int64_t)I_AT(d->value_lookup, d->value_lookup_len, d->p0) + index);
        I_AT(output, olen, bufferStartPos) = code;
        bufferStartPos++;
        if (code > 0) d->low += I_AT(d->summed_probabilities, d->summed_len, p0_index + code - 1) * mult;
        d->high = d->low + I_AT(d->probabilities, d->probabilities_len, p0_index + code) * mult - 1;
        wps->crc += shl32(wps->crc, 1) + code;
        if ((wps->wphdr.flags & MONO_DATA) > 0)
            d->p0 = code & (d->history_bins - 1);
        else {
            d->p0 = d->p1;
            d->p1 = code & (d->history_bins - 1);
        }
        while (((d->high ^ d->low) & 0xFF000000u) == 0 && d->byteptr < d->data_len) {
            d->value = (d->value << 8) | d->data[d->byteptr];
            d->byteptr++;
            d->high = (d->high << 8) | 0xFF;
            d->low <<= 8;
        }
    }
    return sample_count;
}

static void init_ptable(int32_t *table, int rate_i, int rate_s) /* DsdUtils.cs:321-341 */
{
    int value = 0x808000, rate = rate_i << 8, c, i;
    for (c = (rate + 128) >> 8; c > 0; c--) value += (DOWN - value) >> DECAY;
    for (i = 0; i < PTABLE_BINS / 2; ++i) {
        table[i] = value;
        table[PTABLE_BINS - 1 - i] = 0x100ffff - value;
        if (value > 0x010000) {
            rate += (rate * rate_s + 128) >> 8;
            for (c = (rate + 64) >> 7; c > 0; c--) value += (DOWN - value) >> DECAY;
        }
    }
}

static int init_dsd_block_high(WavpackStream *wps) /* DsdUtils.cs:343-389 */
{
    dsds *d = &wps->dsd;
    uint32_t flags = wps->wphdr.flags;
    int channel, rate_i, rate_s, i;
    if (d->data_len - d->byteptr < ((flags & MONO_DATA) > 0 ? 13 : 20)) return 0;
    rate_i = d->data[d->byteptr++];
    rate_s = d->data[d->byteptr++];
    if (rate_s != RATE_S) return 0;
    if (d->ptable == NULL) d->ptable = (int32_t *)calloc(PTABLE_BINS, sizeof(int32_t));
    if (d->filters == NULL) d->filters = (DSDfilters *)calloc(2, sizeof(DSDfilters));
    init_ptable(d->ptable, rate_i, rate_s);
    for (channel = 0; channel < ((flags & MONO_DATA) > 0 ? 1 : 2); ++channel) {
        DSDfilters *sp = &d->filters[channel];
        sp->filter1 = d->data[d->byteptr++] << (PRECISION - 8);
        sp->filter2 = d->data[d->byteptr++] << (PRECISION - 8);
        sp->filter3 = d->data[d->byteptr++] << (PRECISION - 8);
        sp->filter4 = d->data[d->byteptr++] << (PRECISION - 8);
        sp->filter5 = d->data[d->byteptr++] << (PRECISION - 8);
        sp->filter6 = 0;
        sp->factor = d->data[d->byteptr++];
        sp->factor |= d->data[d->byteptr++] << 8;
        sp->factor = (int32_t)((uint32_t)sp->factor << 16) >> 16;
    }
    d->high = 0xFFFFFFFFu;
    d->low = 0x0;
    for (i = 4; i > 0; i--) {
        d->value = (d->value << 8) | d->data[d->byteptr];
        d->byteptr++;
    }
    d->ready = 1;
    return 1;
}

static int64_t decode_high(WavpackStream *wps, int32_t *output, int64_t olen, int64_t sample_count,
                           int bufferStartPos) /* DsdUtils.cs:391-493 */
{
    dsds *d = &wps->dsd;
    int64_t total_samples = sample_count;
    int stereo = (wps->wphdr.flags & MONO_DATA) > 0 ? 0 : 1;
    DSDfilters *sp = d->filters;
    while (total_samples-- > 0) {
        int bitcount = 8;
        sp[0].value = sp[0].filter1 - sp[0].filter5 + ((sp[0].filter6 * sp[0].factor) >> 2);
        if (stereo) sp[1].value = sp[1].filter1 - sp[1].filter5 + ((sp[1].filter6 * sp[1].factor) >> 2);
        while (bitcount-- > 0) {
            for (int ch = 0; ch < 1 + stereo; ch++) {
                DSDfilters *f = &sp[ch];
                int pp = (f->value >> (PRECISION - PRECISION_USE)) & PTABLE_MASK;
                uint32_t split = d->low + ((d->high - d->low) >> 8) * ((uint32_t)d->ptable[pp] >> 16);
                if (d->value <= split) {
                    d->high = split;
                    d->ptable[pp] += (UP - d->ptable[pp]) >> DECAY;
                    f->filter0 = -1;
                } else {
                    d->low = split + 1;
                    d->ptable[pp] += (DOWN - d->ptable[pp]) >> DECAY;
                    f->filter0 = 0;
                }
                while (((d->high ^ d->low) & 0xFF000000u) == 0 && d->byteptr < d->data_len) {
                    d->value = (d->value << 8) | d->data[d->byteptr];
                    d->byteptr++;
                    d->high = (d->high << 8) | 0xFF;
                    d->low <<= 8;
                }
                f->value += f->filter6 * 8;
                f->bytei = shl32(f->bytei, 1) | (f->filter0 & 1);
                f->factor += (((f->value ^ f->filter0) >> 31) | 1) & ((f->value ^ (f->value - (f->filter6 * 16))) >> 31);
                f->filter1 += ((f->filter0 & VALUE_ONE) - f->filter1) >> 6;
                f->filter2 += ((f->filter0 & VALUE_ONE) - f->filter2) >> 4;
                f->filter3 += (f->filter2 - f->filter3) >> 4;
                f->filter4 += (f->filter3 - f->filter4) >> 4;
                f->value = (f->filter4 - f->filter5) >> 4;
                f->filter5 += f->value;
                f->filter6 += (f->value - f->filter6) >> 3;
                f->value = f->filter1 - f->filter5 + ((f->filter6 * f->factor) >> 2);
            }
        }
        int v0 = sp[0].bytei & 0xFF;
        I_AT(output, olen, bufferStartPos) = v0;
        bufferStartPos++;
        wps->crc += shl32(wps->crc, 1) + v0;
        sp[0].factor -= (sp[0].factor + 512) >> 10;
        if (stereo) {
            int v1 = sp[1].bytei & 0xFF;
            I_AT(output, olen, bufferStartPos) = v1;
            bufferStartPos++;
            wps->crc += shl32(wps->crc, 1) + v1;
            sp[1].factor -= (sp[1].factor + 512) >> 10;
        }
    }
    return sample_count;
}

static int init_dsd_block(wvo_ctx *wpc, WavpackMetadata *wpmd) /* DsdUtils.cs:17-54 */
{
    WavpackStream *wps = &wpc->stream;
    int len;
    if (wpmd->byte_length < 2 || B_AT(wpmd->data, wpmd->data_len, 0) > 31) return 0;
    uint8_t *d = copy_data(wpmd, &len);
    if (!d) return 0;
    dsd_release(wpc, &wps->dsd); /* `new dsds()` */
    wps->dsd.data = d;
    wps->dsd.data_len = len;
    wpc->dsd_multiplier = 1u << (wps->dsd.data[wps->dsd.byteptr++] & 31);
    wps->dsd.mode = B_AT(wps->dsd.data, wps->dsd.data_len, wps->dsd.byteptr);
    wps->dsd.byteptr++;
    if (wps->dsd.mode == 0) {
        if ((int64_t)(wps->dsd.data_len - wps->dsd.byteptr) !=
            (int64_t)wps->wphdr.block_samples * ((wps->wphdr.flags & MONO_DATA) > 0 ? 1 : 2))
            return 0;
        wps->dsd.ready = 1;
        return 1;
    } else if (wps->dsd.mode == 1)
        return init_dsd_block_fast(wps);
    else if (wps->dsd.mode == 3)
        return init_dsd_block_high(wps);
    return 0;
}

static int64_t unpack_dsd_samples(wvo_ctx *wpc, int32_t *buffer, int64_t blen, int64_t sample_count,
                                  int bufferStartPos) /* DsdUtils.cs:56-136 */
{
    WavpackStream *wps = &wpc->stream;
    uint32_t flags = wps->wphdr.flags;
    if (wps->sample_index + sample_count > wps->wphdr.block_index + wps->wphdr.block_samples &&
        (wps->wphdr.block_index + wps->wphdr.block_samples - wps->sample_index) < sample_count)
        sample_count = wps->wphdr.block_index + wps->wphdr.block_samples - wps->sample_index;
    if (wps->wphdr.block_index > wps->sample_index || wps->wphdr.block_samples < sample_count) wps->mute_error = 1;
    if (!wps->mute_error) {
        if (wps->dsd.mode == 0) {
            int64_t total = sample_count * ((flags & MONO_DATA) > 0 ? 1 : 2);
            if (wps->dsd.data_len - wps->dsd.byteptr < total) total = wps->dsd.data_len - wps->dsd.byteptr;
            while (total-- > 0) {
                int v = I_AT(wps->dsd.data, wps->dsd.data_len, wps->dsd.byteptr);
                wps->dsd.byteptr++;
                I_AT(buffer, blen, bufferStartPos) = v;
                bufferStartPos++;
                wps->crc += shl32(wps->crc, 1) + v;
            }
        } else if (wps->dsd.mode == 1) {
            if (decode_fast(wps, buffer, blen, sample_count, bufferStartPos) == 0) wps->mute_error = 1;
        } else if (wps->dsd.mode == 3) {
            if (decode_high(wps, buffer, blen, sample_count, bufferStartPos) == 0) wps->mute_error = 1;
        } else
            wps->mute_error = 1;
        if (wps->sample_index + sample_count == wps->wphdr.block_index + wps->wphdr.block_samples &&
            !wps->mute_error && wps->crc != wps->wphdr.crc)
            wps->mute_error = 1;
    }
    if (wps->mute_error) {
        int64_t samples_to_null;
        if (wpc->reduced_channels == 1 || wpc->config.num_channels == 1 || (flags & MONO_FLAG) > 0)
            samples_to_null = sample_count;
        else
            samples_to_null = sample_count * 2;
        while (samples_to_null > 0) I_AT(buffer, blen, --samples_to_null) = 0x55;
        wps->sample_index += sample_count;
        return sample_count;
    }
    if ((flags & FALSE_STEREO) > 0) {
        int dest_idx = (int)sample_count * 2, src_idx = (int)sample_count, c = (int)sample_count;
        while (c-- > 0) {
            src_idx--;
            int32_t v = I_AT(buffer, blen, src_idx + bufferStartPos);
            I_AT(buffer, blen, --dest_idx + bufferStartPos) = v;
            I_AT(buffer, blen, --dest_idx + bufferStartPos) = v;
        }
    }
    wps->sample_index += sample_count;
    return sample_count;
}

/* ------------------------------------------------------------------ */
/* MetadataUtils.cs                                                    */
/* ------------------------------------------------------------------ */
static int read_metadata_buff(wvo_ctx *wpc, WavpackMetadata *wpmd) /* MetadataUtils.cs:15-109 */
{
    int t;
    uint8_t tchar;
    if (wpmd->bytecount >= wpc->stream.wphdr.ckSize) return 0;
    if ((t = rd_byte(&wpc->infile)) < 0) { wpmd->error = 1; return 0; }
    wpmd->id = (uint8_t)t;
    if ((t = rd_byte(&wpc->infile)) < 0) { wpmd->error = 1; return 0; }
    tchar = (uint8_t)t;
    wpmd->bytecount += 2;
    wpmd->byte_length = tchar << 1;
    if ((wpmd->id & ID_LARGE) != 0) {
        wpmd->id &= (uint8_t)~ID_LARGE;
        if ((t = rd_byte(&wpc->infile)) < 0) { wpmd->error = 1; return 0; }
        wpmd->byte_length += t << 9;
        if ((t = rd_byte(&wpc->infile)) < 0) { wpmd->error = 1; return 0; }
        wpmd->byte_length += t << 17;
        wpmd->bytecount += 2;
    }
    int bytes_to_read = wpmd->byte_length;
    if ((wpmd->id & ID_ODD_SIZE) != 0) {
        wpmd->id &= (uint8_t)~ID_ODD_SIZE;
        wpmd->byte_length--;
    }
    if (wpmd->byte_length == 0) {
        wpmd->hasdata = 0;
        return 1;
    }
    wpmd->bytecount += bytes_to_read;
    if (bytes_to_read > 0) {
        if (wpmd->data_is_large) grave(wpc, wpmd->data);
        wpmd->data = wpc->read_buffer;
        wpmd->data_len = BITSTREAM_BUFFER_SIZE;
        wpmd->data_is_large = 0;
        if (bytes_to_read > wpmd->data_len) {
            wpmd->data = (uint8_t *)calloc((size_t)bytes_to_read, 1);
            wpmd->data_len = bytes_to_read;
            wpmd->data_is_large = 1;
        }
        if (rd_read(&wpc->infile, wpmd->data, bytes_to_read) != bytes_to_read) {
            wpmd->hasdata = 0;
            return 0;
        }
        wpmd->hasdata = 1;
    }
    return 1;
}

static int process_metadata(wvo_ctx *wpc, WavpackMetadata *wpmd) /* MetadataUtils.cs:111-192 */
{
    WavpackStream *wps = &wpc->stream;
    switch (wpmd->id) {
    case ID_DUMMY: return 1;
    case ID_DECORR_TERMS: return read_decorr_terms(wps, wpmd);
    case ID_DECORR_WEIGHTS: return read_decorr_weights(wps, wpmd);
    case ID_DECORR_SAMPLES: return read_decorr_samples(wps, wpmd);
    case ID_ENTROPY_VARS: return read_entropy_vars(wps, wpmd);
    case ID_HYBRID_PROFILE: return read_hybrid_profile(wps, wpmd);
    case ID_SHAPING_WEIGHTS: return 1;
    case ID_FLOAT_INFO: return read_float_info(wps, wpmd);
    case ID_INT32_INFO: return read_int32_info(wps, wpmd);
    case ID_CHANNEL_INFO: return read_channel_info(wpc, wpmd);
    case ID_CONFIG_BLOCK: return read_config_info(wpc, wpmd);
    case ID_SAMPLE_RATE: return read_sample_rate(wpc, wpmd);
    case ID_WV_BITSTREAM: return init_wv_bitstream(wpc, wpmd);
    case ID_WVC_BITSTREAM: return init_wvc_bitstream(wpc, wpmd);
    case ID_WVX_BITSTREAM:
    case ID_WVX_NEW_BITSTREAM: return init_wvx_bitstream(wpc, wpmd);
    case ID_DSD_BLOCK: return init_dsd_block(wpc, wpmd);
    case ID_NEW_CONFIG_BLOCK: return read_new_config_info(wpc, wpmd);
    case ID_RIFF_HEADER:
    case ID_ALT_HEADER: return read_header_md(wpc, wpmd, 0);
    case ID_RIFF_TRAILER:
    case ID_ALT_TRAILER: return read_header_md(wpc, wpmd, 1);
    case ID_ALT_EXTENSION:
        if (wpmd->byte_length < 0 || wpmd->byte_length > wpmd->data_len) cs_throw(WVO_EXC_INDEX);
        return 1;
    case ID_BLOCK_CHECKSUM: wpc->five = 1; return 1;
    default:
        if ((wpmd->id & ID_OPTIONAL_DATA) != 0) return 1;
        return 0;
    }
}

/* ------------------------------------------------------------------ */
/* UnpackUtils.cs: unpack_init / unpack_samples / decorr / fixup / crc */
/* ------------------------------------------------------------------ */
static int unpack_init(wvo_ctx *wpc) /* UnpackUtils.cs:24-68 */
{
    WavpackStream *wps = &wpc->stream;
    WavpackMetadata wpmd;
    memset(&wpmd, 0, sizeof(wpmd));
    wpmd.bytecount = 24;
    grave_flush(wpc);

    if (wps->wphdr.block_samples > 0 && wps->wphdr.block_index != 0xFFFFFFFFLL)
        wps->sample_index = wps->wphdr.block_index;
    wps->mute_error = 0;
    wps->crc = wps->crc_x = -1;
    wps->wvbits.sr = 0;

    while (read_metadata_buff(wpc, &wpmd) == 1) {
        if (process_metadata(wpc, &wpmd) == 0) {
            snprintf(wpc->msgbuf, sizeof(wpc->msgbuf), "invalid metadata id %d", wpmd.id);
            wpc->error_message = wpc->msgbuf;
            if (wpmd.data_is_large) grave(wpc, wpmd.data);
            return 0;
        }
    }
    if (wpmd.data_is_large) grave(wpc, wpmd.data);
    if (wpmd.bytecount != wps->wphdr.ckSize) {
        wpc->error_message = "invalid reading WavPack metadata block";
        return 0;
    }
    if ((wps->wphdr.block_samples != 0 && (wps->wphdr.flags & DSD_FLAG) > 0)
            ? !wps->dsd.ready
            : (!wps->wvbits.valid || wps->wvbits.end == 0)) {
        wpc->error_message = "invalid WavPack file";
        return 0;
    }
    if (wps->wphdr.block_samples != 0) {
        if ((wps->wphdr.flags & INT32_DATA) != 0 && wps->int32_sent_bits != 0 && !wps->wvxbits.valid)
            wpc->lossy_blocks = 1;
        if ((wps->wphdr.flags & FLOAT_DATA) != 0 &&
            (wps->float_flags & (FLOAT_EXCEPTIONS | FLOAT_ZEROS_SENT | FLOAT_SHIFT_SENT | FLOAT_SHIFT_SAME)) != 0)
            wpc->lossy_blocks = 1;
    }
    return 1;
}

/* tiny helpers for the stereo pass weight update (UnpackUtils.cs:700-930) */
#define UPD(w, s, b)                        \
    do {                                    \
        if ((s) != 0 && (b) != 0) {         \
            if (((s) ^ (b)) < 0)            \
                (w) -= delta;               \
            else                            \
                (w) += delta;               \
        }                                   \
    } while (0)
#define APPLY(w, s) ((int32_t)(((int64_t)(w) * (int64_t)(s) + 512) >> 10))
/* negative-term clamp (UnpackUtils.cs:757-765) */
#define UPDC(w, s, b)                                                            \
    do {                                                                         \
        if (((s) ^ (b)) < 0) {                                                   \
            if ((s) != 0 && (b) != 0 && ((w) -= delta) < -1024) (w) = ((w) < 0) ? -1024 : 1024; \
        } else {                                                                 \
            if ((s) != 0 && (b) != 0 && ((w) += delta) > 1024) (w) = ((w) < 0) ? -1024 : 1024; \
        }                                                                        \
    } while (0)

static void decorr_stereo_pass(decorr_pass *dpp, int32_t *buf, int64_t blen, int64_t sample_count,
                               int buf_idx) /* UnpackUtils.cs:688-944 */
{
    int delta = dpp->delta;
    int weight_A = dpp->weight_A, weight_B = dpp->weight_B;
    int sam_A, sam_B, m, k;
    int64_t p, end = buf_idx + sample_count * 2;
#define BI(i) I_AT(buf, blen, (i))
    switch (dpp->term) {
    case 17:
        for (p = buf_idx; p < end; p += 2) {
            sam_A = 2 * dpp->samples_A[0] - dpp->samples_A[1];
            dpp->samples_A[1] = dpp->samples_A[0];
            dpp->samples_A[0] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[0];
            sam_A = 2 * dpp->samples_B[0] - dpp->samples_B[1];
            dpp->samples_B[1] = dpp->samples_B[0];
            dpp->samples_B[0] = APPLY(weight_B, sam_A) + BI(p + 1);
            UPD(weight_B, sam_A, BI(p + 1));
            BI(p + 1) = dpp->samples_B[0];
        }
        break;
    case 18:
        for (p = buf_idx; p < end; p += 2) {
            sam_A = (3 * dpp->samples_A[0] - dpp->samples_A[1]) >> 1;
            dpp->samples_A[1] = dpp->samples_A[0];
            dpp->samples_A[0] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[0];
            sam_A = (3 * dpp->samples_B[0] - dpp->samples_B[1]) >> 1;
            dpp->samples_B[1] = dpp->samples_B[0];
            dpp->samples_B[0] = APPLY(weight_B, sam_A) + BI(p + 1);
            UPD(weight_B, sam_A, BI(p + 1));
            BI(p + 1) = dpp->samples_B[0];
        }
        break;
    case -1:
        for (p = buf_idx; p < end; p += 2) {
            sam_A = BI(p) + APPLY(weight_A, dpp->samples_A[0]);
            UPDC(weight_A, dpp->samples_A[0], BI(p));
            BI(p) = sam_A;
            dpp->samples_A[0] = BI(p + 1) + APPLY(weight_B, sam_A);
            UPDC(weight_B, sam_A, BI(p + 1));
            BI(p + 1) = dpp->samples_A[0];
        }
        break;
    case -2:
        for (p = buf_idx; p < end; p += 2) {
            sam_B = BI(p + 1) + APPLY(weight_B, dpp->samples_B[0]);
            UPDC(weight_B, dpp->samples_B[0], BI(p + 1));
            BI(p + 1) = sam_B;
            dpp->samples_B[0] = BI(p) + APPLY(weight_A, sam_B);
            UPDC(weight_A, sam_B, BI(p));
            BI(p) = dpp->samples_B[0];
        }
        break;
    case -3:
        for (p = buf_idx; p < end; p += 2) {
            sam_A = BI(p) + APPLY(weight_A, dpp->samples_A[0]);
            UPDC(weight_A, dpp->samples_A[0], BI(p));
            sam_B = BI(p + 1) + APPLY(weight_B, dpp->samples_B[0]);
            UPDC(weight_B, dpp->samples_B[0], BI(p + 1));
            BI(p) = dpp->samples_B[0] = sam_A;
            BI(p + 1) = dpp->samples_A[0] = sam_B;
        }
        break;
    default:
        for (m = 0, k = dpp->term & (MAX_TERM - 1), p = buf_idx; p < end; p += 2) {
            sam_A = dpp->samples_A[m];
            dpp->samples_A[k] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[k];
            sam_A = dpp->samples_B[m];
            dpp->samples_B[k] = APPLY(weight_B, sam_A) + BI(p + 1);
            UPD(weight_B, sam_A, BI(p + 1));
            BI(p + 1) = dpp->samples_B[k];
            m = (m + 1) & (MAX_TERM - 1);
            k = (k + 1) & (MAX_TERM - 1);
        }
        if (m != 0) {
            int32_t tmp[MAX_TERM];
            memcpy(tmp, dpp->samples_A, sizeof(tmp));
            for (k = 0; k < MAX_TERM; k++, m++) dpp->samples_A[k] = tmp[m & (MAX_TERM - 1)];
            memcpy(tmp, dpp->samples_B, sizeof(tmp));
            for (k = 0; k < MAX_TERM; k++, m++) dpp->samples_B[k] = tmp[m & (MAX_TERM - 1)];
        }
        break;
    }
    dpp->weight_A = (int16_t)weight_A;
    dpp->weight_B = (int16_t)weight_B;
}

/* weight update of the *_cont loops: w += (((a ^ b) >> 30) | 1) * delta (UnpackUtils.cs:965) */
#define UPD30(w, a, b)                                                    \
    do {                                                                  \
        if ((a) != 0 && (b) != 0) (w) += ((((a) ^ (b)) >> 30) | 1) * delta; \
    } while (0)

static void decorr_stereo_pass_cont(decorr_pass *dpp, int32_t *buf, int64_t blen, int64_t sample_count,
                                    int buf_idx) /* UnpackUtils.cs:946-1154 */
{
    int delta = dpp->delta, weight_A = dpp->weight_A, weight_B = dpp->weight_B;
    int64_t tptr;
    int sam_A, sam_B, k, i, v;
    int64_t bi = buf_idx, end = buf_idx + sample_count * 2;
    switch (dpp->term) {
    case 17:
        for (bi = buf_idx; bi < end; bi += 2) {
            sam_A = 2 * BI(bi - 2) - BI(bi - 4);
            sam_B = BI(bi);
            BI(bi) = APPLY(weight_A, sam_A) + sam_B;
            UPD30(weight_A, sam_A, sam_B);
            sam_A = 2 * BI(bi - 1) - BI(bi - 3);
            sam_B = BI(bi + 1);
            BI(bi + 1) = APPLY(weight_B, sam_A) + sam_B;
            UPD30(weight_B, sam_A, sam_B);
        }
        dpp->samples_B[0] = BI(bi - 1);
        dpp->samples_A[0] = BI(bi - 2);
        dpp->samples_B[1] = BI(bi - 3);
        dpp->samples_A[1] = BI(bi - 4);
        break;
    case 18:
        for (bi = buf_idx; bi < end; bi += 2) {
            sam_A = (3 * BI(bi - 2) - BI(bi - 4)) >> 1;
            sam_B = BI(bi);
            BI(bi) = APPLY(weight_A, sam_A) + sam_B;
            UPD30(weight_A, sam_A, sam_B);
            sam_A = (3 * BI(bi - 1) - BI(bi - 3)) >> 1;
            sam_B = BI(bi + 1);
            BI(bi + 1) = APPLY(weight_B, sam_A) + sam_B;
            UPD30(weight_B, sam_A, sam_B);
        }
        dpp->samples_B[0] = BI(bi - 1);
        dpp->samples_A[0] = BI(bi - 2);
        dpp->samples_B[1] = BI(bi - 3);
        dpp->samples_A[1] = BI(bi - 4);
        break;
    case -1:
        for (bi = buf_idx; bi < end; bi += 2) {
            v = APPLY(weight_A, BI(bi - 1));
            sam_A = BI(bi);
            BI(bi) = v + sam_A;
            UPDC(weight_A, BI(bi - 1), sam_A);
            v = APPLY(weight_B, BI(bi));
            sam_A = BI(bi + 1);
            BI(bi + 1) = v + sam_A;
            UPDC(weight_B, BI(bi), sam_A);
        }
        dpp->samples_A[0] = BI(bi - 1);
        break;
    case -2:
        for (bi = buf_idx; bi < end; bi += 2) {
            v = APPLY(weight_B, BI(bi - 2));
            sam_A = BI(bi + 1);
            BI(bi + 1) = v + sam_A;
            UPDC(weight_B, BI(bi - 2), sam_A);
            v = APPLY(weight_A, BI(bi + 1));
            sam_A = BI(bi);
            BI(bi) = v + sam_A;
            UPDC(weight_A, BI(bi + 1), sam_A);
        }
        dpp->samples_B[0] = BI(bi - 2);
        break;
    case -3:
        for (bi = buf_idx; bi < end; bi += 2) {
            v = APPLY(weight_A, BI(bi - 1));
            sam_A = BI(bi);
            BI(bi) = v + sam_A;
            UPDC(weight_A, BI(bi - 1), sam_A);
            v = APPLY(weight_B, BI(bi - 2));
            sam_A = BI(bi + 1);
            BI(bi + 1) = v + sam_A;
            UPDC(weight_B, BI(bi - 2), sam_A);
        }
        dpp->samples_A[0] = BI(bi - 1);
        dpp->samples_B[0] = BI(bi - 2);
        break;
    default:
        tptr = buf_idx - (dpp->term * 2);
        for (bi = buf_idx; bi < end; bi += 2) {
            v = APPLY(weight_A, BI(tptr));
            sam_A = BI(bi);
            BI(bi) = v + sam_A;
            UPD30(weight_A, BI(tptr), sam_A);
            v = APPLY(weight_B, BI(tptr + 1));
            sam_A = BI(bi + 1);
            BI(bi + 1) = v + sam_A;
            UPD30(weight_B, BI(tptr + 1), sam_A);
            tptr += 2;
        }
        bi--;
        for (k = dpp->term - 1, i = 8; i > 0; k--) {
            i--;
            dpp->samples_B[k & (MAX_TERM - 1)] = BI(bi);
            bi--;
            dpp->samples_A[k & (MAX_TERM - 1)] = BI(bi);
            bi--;
        }
        break;
    }
    dpp->weight_A = (int16_t)weight_A;
    dpp->weight_B = (int16_t)weight_B;
}

static void decorr_mono_pass(decorr_pass *dpp, int32_t *buf, int64_t blen, int64_t sample_count,
                             int buf_idx) /* UnpackUtils.cs:1156-1240 */
{
    int delta = dpp->delta, weight_A = dpp->weight_A;
    int sam_A, m, k;
    int64_t p, end = buf_idx + sample_count;
    switch (dpp->term) {
    case 17:
        for (p = buf_idx; p < end; p++) {
            sam_A = 2 * dpp->samples_A[0] - dpp->samples_A[1];
            dpp->samples_A[1] = dpp->samples_A[0];
            dpp->samples_A[0] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[0];
        }
        break;
    case 18:
        for (p = buf_idx; p < end; p++) {
            sam_A = (3 * dpp->samples_A[0] - dpp->samples_A[1]) >> 1;
            dpp->samples_A[1] = dpp->samples_A[0];
            dpp->samples_A[0] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[0];
        }
        break;
    default:
        for (m = 0, k = dpp->term & (MAX_TERM - 1), p = buf_idx; p < end; p++) {
            sam_A = dpp->samples_A[m];
            dpp->samples_A[k] = APPLY(weight_A, sam_A) + BI(p);
            UPD(weight_A, sam_A, BI(p));
            BI(p) = dpp->samples_A[k];
            m = (m + 1) & (MAX_TERM - 1);
            k = (k + 1) & (MAX_TERM - 1);
        }
        if (m != 0) {
            int32_t tmp[MAX_TERM];
            memcpy(tmp, dpp->samples_A, sizeof(tmp));
            for (k = 0; k < MAX_TERM; k++, m++) dpp->samples_A[k] = tmp[m & (MAX_TERM - 1)];
        }
        break;
    }
    dpp->weight_A = (int16_t)weight_A;
}

static void fixup_samples(WavpackStream *wps, int32_t *buf, int64_t blen, int64_t sample_count,
                          int bufferStartPos) /* UnpackUtils.cs:1251-1404 */
{
    int64_t flags = wps->wphdr.flags;
    int lossy_flag = (flags & HYBRID_FLAG) > 0;
    int shift = (int)((flags & SHIFT_MASK) >> SHIFT_LSB);

    if ((flags & FLOAT_DATA) > 0) {
        float_values(wps, buf, blen, (flags & MONO_FLAG) > 0 ? sample_count : sample_count * 2, bufferStartPos);
        return;
    }
    if ((flags & INT32_DATA) > 0) {
        int64_t count = (flags & MONO_FLAG) > 0 ? sample_count : sample_count * 2;
        int sent_bits = wps->int32_sent_bits, zeros = wps->int32_zeros;
        int ones = wps->int32_ones, dups = wps->int32_dups;
        uint32_t data, mask = (uint32_t)shl32(1, sent_bits) - 1u;
        int64_t bc = bufferStartPos;
        if (wps->wvxbits.valid) {
            int max_width = wps->int32_max_width;
            int crc = wps->crc_x;
            while (count-- > 0) {
                int32_t *x = &BI(bc);
                if (sent_bits > 0) {
                    if (max_width > 0) {
                        int pvalue = *x < 0 ? ~*x : *x;
                        int width = count_bits(pvalue) + sent_bits;
                        int bits_to_read = sent_bits;
                        if (width <= max_width || (bits_to_read -= width - max_width) > 0) {
                            data = (uint32_t)getbits(bits_to_read, &wps->wvxbits) & mask;
                            *x = shl32((int32_t)((uint32_t)shl32(*x, bits_to_read) | data), sent_bits - bits_to_read);
                        } else
                            *x = shl32(*x, sent_bits);
                    } else {
                        data = (uint32_t)(getbits(sent_bits, &wps->wvxbits) & mask);
                        *x = (int32_t)(((uint32_t)shl32(*x, sent_bits)) | data);
                    }
                }
                if (zeros != 0)
                    *x = shl32(*x, zeros);
                else if (ones != 0)
                    *x = shl32(*x + 1, ones) - 1;
                else if (dups != 0)
                    *x = shl32(*x + (*x & 1), dups) - (*x & 1);
                crc = crc * 9 + (*x & 0xffff) * 3 + ((*x >> 16) & 0xffff);
                bc++;
            }
            wps->crc_x = crc;
        } else if (sent_bits == 0 && (zeros + ones + dups) != 0) {
            while (lossy_flag && (flags & BYTES_STORED) == 3 && shift < 8) {
                if (zeros > 0)
                    zeros--;
                else if (ones > 0)
                    ones--;
                else if (dups > 0)
                    dups--;
                else
                    break;
                shift++;
            }
            while (count-- > 0) {
                int32_t *x = &BI(bc);
                if (zeros != 0)
                    *x = shl32(*x, zeros);
                else if (ones != 0)
                    *x = shl32(*x + 1, ones) - 1;
                else if (dups != 0)
                    *x = shl32(*x + (*x & 1), dups) - (*x & 1);
                bc++;
            }
        } else
            shift += zeros + sent_bits + ones + dups;
    }
    shift &= 0x1f;
    if (lossy_flag) {
        int min_value, max_value, min_shifted, max_shifted;
        int64_t bc = bufferStartPos;
        switch (flags & BYTES_STORED) {
        case 0:
            min_shifted = shl32(min_value = sar32(-128, shift), shift);
            max_shifted = shl32(max_value = sar32(127, shift), shift);
            break;
        case 1:
            min_shifted = shl32(min_value = sar32(-32768, shift), shift);
            max_shifted = shl32(max_value = sar32(32767, shift), shift);
            break;
        case 2:
            min_shifted = shl32(min_value = sar32(-8388608, shift), shift);
            max_shifted = shl32(max_value = sar32(8388607, shift), shift);
            break;
        default:
            min_shifted = shl32(min_value = (int32_t)shr32u(0x80000000u, shift), shift);
            max_shifted = shl32(max_value = sar32(0x7FFFFFFF, shift), shift);
            break;
        }
        if ((flags & MONO_FLAG) == 0) sample_count *= 2;
        while (sample_count-- > 0) {
            int32_t *x = &BI(bc);
            if (*x < min_value)
                *x = min_shifted;
            else if (*x > max_value)
                *x = max_shifted;
            else
                *x = shl32(*x, shift);
            bc++;
        }
    } else if (shift != 0) {
        int64_t bc = bufferStartPos;
        if ((flags & MONO_FLAG) == 0) sample_count *= 2;
        while (sample_count-- > 0) {
            int32_t *x = &BI(bc);
            *x = shl32(*x, shift);
            bc++;
        }
    }
}

static int check_crc_error(wvo_ctx *wpc) /* UnpackUtils.cs:1414-1421 */
{
    WavpackStream *wps = &wpc->stream;
    return wps->crc != wps->wphdr.crc ||
           ((wps->wphdr.flags & FLOAT_DATA) == 0 && wps->wvxbits.valid && wps->crc_x != wps->crc_mvx);
}

static int64_t unpack_samples(wvo_ctx *wpc, int32_t *buf, int64_t blen, int64_t sample_count,
                              int bufferStartPos) /* UnpackUtils.cs:510-686 */
{
    WavpackStream *wps = &wpc->stream;
    int64_t flags = wps->wphdr.flags;
    int64_t i;
    int crc = wps->crc;
    int mute_limit = (int)((1LL << (int)((flags & MAG_MASK) >> MAG_LSB)) + 2);
    int tcount;
    int64_t bcnt;

    if (wps->sample_index + sample_count > wps->wphdr.block_index + wps->wphdr.block_samples)
        sample_count = wps->wphdr.block_index + wps->wphdr.block_samples - wps->sample_index;

    if (wps->mute_error) {
        int64_t tempc = (flags & MONO_FLAG) > 0 ? sample_count : 2 * sample_count;
        bcnt = bufferStartPos;
        while (tempc-- > 0) BI(bcnt++) = 0;
        wps->sample_index += sample_count;
        return sample_count;
    }
    if ((flags & HYBRID_FLAG) > 0) mute_limit *= 2;

    if ((flags & MONO_DATA) > 0) {
        i = get_words(sample_count, flags, &wps->w, &wps->wvbits, buf, blen, bufferStartPos);
        for (tcount = 0; tcount < wps->num_terms; tcount++)
            decorr_mono_pass(&I_AT(wps->decorr_passes, MAX_NTERMS, tcount), buf, blen, sample_count, bufferStartPos);
        int crclimit = (int)(sample_count + bufferStartPos);
        for (int q = bufferStartPos; q < crclimit; q++) {
            int bf_i = BI(q);
            int bf_abs = bf_i < 0 ? -bf_i : bf_i;
            if (bf_abs > mute_limit) {
                i = q; /* absolute index: quirk B-6 */
                break;
            }
            crc = crc * 3 + bf_i;
        }
    } else {
        i = get_words(sample_count, flags, &wps->w, &wps->wvbits, buf, blen, bufferStartPos);
        if (sample_count < 16) {
            for (tcount = 0; tcount < wps->num_terms; tcount++)
                decorr_stereo_pass(&I_AT(wps->decorr_passes, MAX_NTERMS, tcount), buf, blen, sample_count, bufferStartPos);
        } else {
            for (tcount = 0; tcount < wps->num_terms; tcount++) {
                decorr_pass *dpp = &I_AT(wps->decorr_passes, MAX_NTERMS, tcount);
                decorr_stereo_pass(dpp, buf, blen, 8, bufferStartPos);
                decorr_stereo_pass_cont(dpp, buf, blen, sample_count - 8, bufferStartPos + 16);
            }
        }
        int joint = (flags & JOINT_STEREO) > 0;
        for (bcnt = 0; bcnt < sample_count * 2; bcnt += 2) {
            int64_t a = bcnt + bufferStartPos;
            if (joint) {
                BI(a + 1) -= BI(a) >> 1;
                BI(a) += BI(a + 1);
            }
            int l = BI(a), r = BI(a + 1);
            int bf_abs = l < 0 ? -l : l;
            int bf1_abs = r < 0 ? -r : r;
            if (bf_abs > mute_limit || bf1_abs > mute_limit) {
                i = bcnt / 2;
                break;
            }
            crc = (crc * 3 + l) * 3 + r;
        }
    }

    if (i != sample_count) {
        int64_t sc = (flags & MONO_FLAG) > 0 ? sample_count : 2 * sample_count;
        bcnt = bufferStartPos;
        while (sc-- > 0) BI(bcnt++) = 0;
        wps->mute_error = 1;
        i = sample_count;
    }

    fixup_samples(wps, buf, blen, i, bufferStartPos);

    if ((flags & FALSE_STEREO) > 0) {
        int dest_idx = (int)i * 2, src_idx = (int)i, c = (int)i;
        while (c-- > 0) {
            src_idx--;
            int32_t v = BI(src_idx + bufferStartPos);
            BI(--dest_idx + bufferStartPos) = v;
            BI(--dest_idx + bufferStartPos) = v;
        }
    }
    wps->sample_index += i;
    wps->crc = crc;
    return i;
}
#undef BI

/* ------------------------------------------------------------------ */
/* WavPackUtils.cs                                                     */
/* ------------------------------------------------------------------ */
static void read_next_header(Reader *infile, WavpackHeader *wphdr) /* WavPackUtils.cs:600-671 */
{
    uint8_t buffer[32];
    int64_t bytes_skipped = 0;
    int bleft = 0, counter;
    while (1) {
        for (int i = 0; i < bleft; i++) buffer[i] = buffer[32 - bleft + i];
        counter = 0;
        int cnt = 32 - bleft;
        if (rd_read(infile, buffer + bleft, cnt) != cnt) {
            wphdr->error = 1;
            return;
        }
        bleft = 32;
        if (buffer[0] == 'w' && buffer[1] == 'v' && buffer[2] == 'p' && buffer[3] == 'k' && (buffer[4] & 1) == 0 &&
            buffer[6] < 16 && buffer[7] == 0 && buffer[9] == 4 && buffer[8] >= (MIN_STREAM_VERS & 0xff) &&
            buffer[8] <= (MAX_STREAM_VERS & 0xff)) {
            wphdr->ckSize = (uint32_t)((buffer[7] << 24) | (buffer[6] << 16) | (buffer[5] << 8) | buffer[4]);
            wphdr->version = (int16_t)((buffer[9] << 8) | buffer[8]);
            wphdr->total_samples = (int64_t)(((uint64_t)buffer[11] << 32) | ((uint64_t)buffer[15] << 24) |
                                             ((uint64_t)buffer[14] << 16) | ((uint64_t)buffer[13] << 8) | buffer[12]);
            wphdr->block_index = (int64_t)(((uint64_t)buffer[10] << 32) | ((uint64_t)buffer[19] << 24) |
                                           ((uint64_t)buffer[18] << 16) | ((uint64_t)buffer[17] << 8) | buffer[16]);
            wphdr->block_samples = (uint32_t)((buffer[23] << 24) | (buffer[22] << 16) | (buffer[21] << 8) | buffer[20]);
            wphdr->flags = (uint32_t)((buffer[27] << 24) | (buffer[26] << 16) | (buffer[25] << 8) | buffer[24]);
            wphdr->crc = (int32_t)(((uint32_t)buffer[31] << 24) | (buffer[30] << 16) | (buffer[29] << 8) | buffer[28]);
            wphdr->error = 0;
            wphdr->stream_position = infile->pos - bleft;
            if (wphdr->average_block_size == 0)
                wphdr->average_block_size = wphdr->ckSize;
            else
                wphdr->average_block_size = (wphdr->average_block_size + wphdr->ckSize) / 2;
            return;
        } else {
            counter++;
            bleft--;
        }
        while (bleft > 0 && buffer[counter] != 'w') {
            counter++;
            bleft--;
        }
        bytes_skipped += counter;
        if (bytes_skipped > 1048576LL) {
            wphdr->error = 1;
            return;
        }
    }
}

static void ctx_init(wvo_ctx *wpc)
{
    memset(wpc, 0, sizeof(*wpc));
    /* `new Bitstream()` for wvbits: non-null, empty 16K buffer, end = 0 */
    wpc->stream.wvbits.valid = 1;
    wpc->stream.wvbits.buf = (uint8_t *)calloc(BITSTREAM_BUFFER_SIZE, 1);
    wpc->stream.wvbits.buf_len = BITSTREAM_BUFFER_SIZE;
}

static wvo_ctx *open_at(const uint8_t *file, size_t len, uint32_t flags, int64_t pos);

wvo_ctx *wvo_open(const uint8_t *file, size_t len, uint32_t flags) /* WavPackUtils.cs:36-120 */
{
    return open_at(file, len, flags, 0);
}

/* WavpackOpenFileInput on a BinaryReader positioned at `pos` (seek re-opens at a block) */
static wvo_ctx *open_at(const uint8_t *file, size_t len, uint32_t flags, int64_t pos)
{
    wvo_ctx *wpc = (wvo_ctx *)malloc(sizeof(wvo_ctx));
    jmp_buf jb, *saved = g_jmp;
    ctx_init(wpc);
    WavpackStream *wps = &wpc->stream;
    wpc->infile.data = file;
    wpc->infile.len = (int64_t)len;
    wpc->infile.pos = pos;
    wpc->total_samples = -1;
    wpc->norm_offset = 0;
    wpc->open_flags = 0;
    g_jmp = &jb;
    if (setjmp(jb)) {
        g_jmp = saved;
        wpc->exception = g_exc;
        wpc->error_message = "exception";
        return wpc;
    }
    while (wps->wphdr.block_samples == 0) {
        read_next_header(&wpc->infile, &wps->wphdr);
        if (wps->wphdr.error) {
            wpc->error_message = "not compatible with this version of WavPack file!";
            g_jmp = saved;
            return wpc;
        }
        if (wps->wphdr.block_samples > 0 && wps->wphdr.total_samples != 0xFFFFFFFFLL)
            wpc->total_samples = wps->wphdr.total_samples;
        if (unpack_init(wpc) == 0) {
            g_jmp = saved;
            return wpc;
        }
    }
    wpc->config.flags = wpc->config.flags & ~0xffLL;
    wpc->config.flags = wpc->config.flags | (wps->wphdr.flags & 0xff);
    wpc->config.bytes_per_sample = (int)((wps->wphdr.flags & BYTES_STORED) + 1);
    wpc->config.float_norm_exp = wps->float_norm_exp;
    wpc->config.bits_per_sample =
        (int)((wpc->config.bytes_per_sample * 8) - ((wps->wphdr.flags & SHIFT_MASK) >> SHIFT_LSB));
    if ((wpc->config.flags & FLOAT_DATA) > 0) {
        wpc->config.bytes_per_sample = 3;
        wpc->config.bits_per_sample = 24;
    }
    if (wpc->config.sample_rate == 0) {
        if (wps->wphdr.block_samples == 0 || (wps->wphdr.flags & SRATE_MASK) == SRATE_MASK)
            wpc->config.sample_rate = 44100;
        else
            wpc->config.sample_rate = sample_rates[(int)((wps->wphdr.flags & SRATE_MASK) >> SRATE_LSB)];
    }
    if (wpc->config.num_channels == 0) {
        wpc->config.num_channels = (wps->wphdr.flags & MONO_FLAG) > 0 ? 1 : 2;
        wpc->config.channel_mask = 0x5 - wpc->config.num_channels;
    }
    if ((flags & OPEN_2CH_MAX) > 0 && (wps->wphdr.flags & FINAL_BLOCK) == 0)
        wpc->reduced_channels = (wps->wphdr.flags & MONO_FLAG) != 0 ? 1 : 2;
    if ((flags & OPEN_2CH_MAX) == 0 && wpc->config.num_channels > 2) {
        wpc->error_message = "only two channels supported!";
        g_jmp = saved;
        return wpc;
    }
    if ((wps->wphdr.flags & DSD_FLAG) != 0) {
        wpc->config.bytes_per_sample = 1;
        wpc->config.bits_per_sample = 8;
    }
    g_jmp = saved;
    return wpc;
}

void wvo_close(wvo_ctx *wpc)
{
    if (!wpc) return;
    WavpackStream *wps = &wpc->stream;
    if (wps->wvbits.valid) free(wps->wvbits.buf);
    if (wps->wvcbits.valid) free(wps->wvcbits.buf);
    if (wps->wvxbits.valid) free(wps->wvxbits.buf);
    dsd_release(wpc, &wps->dsd);
    grave_flush(wpc);
    free(wpc->graveyard);
    free(wpc->header);
    free(wpc->trailer);
    free(wpc);
}

int64_t wvo_unpack_samples(wvo_ctx *wpc, int32_t *buffer, int64_t blen, int64_t samples) /* WavPackUtils.cs:200-282 */
{
    WavpackStream *wps = &wpc->stream;
    int64_t samples_unpacked = 0, samples_to_unpack;
    int num_channels = wpc->config.num_channels;
    int64_t bcounter = 0;
    int buf_idx = 0;
    int bytes_returned = 0;
    jmp_buf jb, *saved = g_jmp;
    g_jmp = &jb;
    if (setjmp(jb)) {
        g_jmp = saved;
        wpc->exception = g_exc;
        return -1;
    }
    while (samples > 0) {
        if (wps->wphdr.block_samples == 0 || (wps->wphdr.flags & INITIAL_BLOCK) == 0 ||
            wps->sample_index >= wps->wphdr.block_index + wps->wphdr.block_samples) {
            read_next_header(&wpc->infile, &wps->wphdr);
            if (wps->wphdr.error) break;
            if (wps->wphdr.block_samples == 0 || wps->sample_index == wps->wphdr.block_index)
                if (unpack_init(wpc) == 0) break;
        }
        if (wps->wphdr.block_samples == 0 || (wps->wphdr.flags & INITIAL_BLOCK) == 0 ||
            wps->sample_index >= wps->wphdr.block_index + wps->wphdr.block_samples)
            continue;
        if (wps->sample_index < wps->wphdr.block_index) {
            samples_to_unpack = wps->wphdr.block_index - wps->sample_index;
            if (samples_to_unpack > samples) samples_to_unpack = samples;
            wps->sample_index += samples_to_unpack;
            samples_unpacked += samples_to_unpack;
            samples -= samples_to_unpack;
            if (wpc->reduced_channels > 0)
                samples_to_unpack *= wpc->reduced_channels;
            else
                samples_to_unpack *= num_channels;
            bcounter = buf_idx;
            while (samples_to_unpack-- > 0) I_AT(buffer, blen, bcounter++) = 0;
            buf_idx = (int)bcounter;
            continue;
        }
        samples_to_unpack = wps->wphdr.block_index + wps->wphdr.block_samples - wps->sample_index;
        if (samples_to_unpack > samples) samples_to_unpack = samples;
        if ((wps->wphdr.flags & DSD_FLAG) > 0)
            unpack_dsd_samples(wpc, buffer, blen, samples_to_unpack, buf_idx);
        else
            unpack_samples(wpc, buffer, blen, samples_to_unpack, buf_idx);
        if (wpc->reduced_channels > 0)
            bytes_returned = (int)(samples_to_unpack * wpc->reduced_channels);
        else
            bytes_returned = (int)(samples_to_unpack * num_channels);
        buf_idx += bytes_returned;
        samples_unpacked += samples_to_unpack;
        samples -= samples_to_unpack;
        if (wps->sample_index == wps->wphdr.block_index + wps->wphdr.block_samples)
            if (check_crc_error(wpc)) wpc->crc_errors++;
        if (wps->sample_index == wpc->total_samples) break;
    }
    g_jmp = saved;
    return samples_unpacked;
}

/* WavpackContext.stream = c.stream: the context adopts the stream of a context
 * opened at a block (its arrays move; the old stream's arrays are released) */
static void adopt_stream(wvo_ctx *wpc, wvo_ctx *c)
{
    WavpackStream *wps = &wpc->stream;
    if (wps->wvbits.valid) free(wps->wvbits.buf);
    if (wps->wvcbits.valid) free(wps->wvcbits.buf);
    if (wps->wvxbits.valid) free(wps->wvxbits.buf);
    dsd_release(wpc, &wps->dsd);
    memcpy(wps, &c->stream, sizeof(*wps));
    memset(&c->stream, 0, sizeof(c->stream));
    wvo_close(c);
}

int wvo_set_sample(wvo_ctx *wpc, int64_t targetSample) /* SetSample -> seek, WavPackUtils.cs:509-594 */
{
    WavpackStream *wps = &wpc->stream;
    jmp_buf jb, *saved = g_jmp;
    g_jmp = &jb;
    if (setjmp(jb)) { /* only IOException is caught inside seek (:590); anything else escapes */
        g_jmp = saved;
        wpc->exception = g_exc;
        return -1;
    }
    if (targetSample >= wpc->total_samples) {
        g_jmp = saved;
        return 0;
    }
    if (targetSample < 0) targetSample = 0;
    int steps = 25;      /* maximum steps to position */
    const int min = 5;   /* min count of block for seek forward by just read header */
    while (steps-- > 0) {
        int64_t seek_pos = wps->wphdr.stream_position;
        if (targetSample <= (int64_t)wps->wphdr.block_samples)
            seek_pos = 0;
        else if (targetSample < wps->wphdr.block_index ||
                 targetSample > wps->wphdr.block_index + (int64_t)wps->wphdr.block_samples) {
            int64_t distance = targetSample - wps->wphdr.block_index;
            distance += distance > 0 ? (-1 * (int64_t)wps->wphdr.block_samples + 1)
                                     : (-2 * (int64_t)wps->wphdr.block_samples + 1);
            if (wps->wphdr.block_samples == 0) cs_throw(WVO_EXC_DIVZERO);
            int64_t blocks = distance / (int64_t)wps->wphdr.block_samples;
            if (blocks >= 0 && blocks <= min)
                seek_pos = -1;
            else
                seek_pos += blocks * wps->wphdr.average_block_size;
            if (seek_pos >= wpc->infile.len) seek_pos = -1;
        }
        if (seek_pos != -1) {
            if (seek_pos < 0) { /* Stream.Seek before the beginning: IOException, caught (:590) */
                g_jmp = saved;
                return 0;
            }
            wpc->infile.pos = seek_pos;
        }
        read_next_header(&wpc->infile, &wps->wphdr);
        if (wps->wphdr.error) continue;
        if (steps == 0 || (targetSample >= wps->wphdr.block_index &&
                           targetSample < wps->wphdr.block_index + (int64_t)wps->wphdr.block_samples)) {
            int64_t index = targetSample - wps->wphdr.block_index;
            wvo_ctx *c = open_at(wpc->infile.data, (size_t)wpc->infile.len, 0, wps->wphdr.stream_position);
            wpc->infile.pos = c->infile.pos; /* one shared BinaryReader */
            if (c->exception) {
                int e = c->exception;
                wvo_close(c);
                cs_throw(e);
            }
            adopt_stream(wpc, c);
            int32_t temp_buf[SAMPLE_BUFFER_SIZE];
            while (index > 0) {
                int64_t toUnpack = SAMPLE_BUFFER_SIZE / wvo_get_reduced_channels(wpc);
                if (index < toUnpack) toUnpack = index;
                g_jmp = saved;
                toUnpack = wvo_unpack_samples(wpc, temp_buf, SAMPLE_BUFFER_SIZE, toUnpack);
                g_jmp = &jb;
                if (toUnpack < 0) { /* the exception escapes SetSample */
                    g_jmp = saved;
                    return -1;
                }
                if (toUnpack == 0) { /* the C# loop never ends */
                    wpc->exception = WVO_EXC_HANG;
                    g_jmp = saved;
                    return -1;
                }
                index -= toUnpack;
            }
            g_jmp = saved;
            return 1;
        }
        if (seek_pos == -1) {
            wpc->infile.pos = wps->wphdr.stream_position + wps->wphdr.ckSize;
            steps--; /* "do not account forward seek by headers" (:586) */
        }
    }
    g_jmp = saved;
    return 0;
}

int64_t wvo_decode_file_from(const uint8_t *file, size_t len, int64_t start, int32_t *out, int64_t out_cap, int chunk,
                             int64_t *crc_errors, int *nch, int *seek_rc)
{
    wvo_ctx *wpc = wvo_open(file, len, 0);
    if (wpc->error_message && wpc->error_message[0]) {
        wvo_close(wpc);
        return -2;
    }
    int ch = wvo_get_reduced_channels(wpc);
    *seek_rc = wvo_set_sample(wpc, start);
    if (*seek_rc < 0) {
        wvo_close(wpc);
        return -3;
    }
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (size_t)chunk * (size_t)ch);
    int64_t total = 0, got, rv = 0;
    while (1) {
        got = wvo_unpack_samples(wpc, tmp, (int64_t)chunk * ch, chunk);
        if (got < 0) { rv = -3; break; }
        if (got > 0) {
            int64_t n = got * ch;
            if ((total * ch + n) <= out_cap) memcpy(out + total * ch, tmp, sizeof(int32_t) * (size_t)n);
            total += got;
        }
        if (got == 0) break;
    }
    if (crc_errors) *crc_errors = wvo_get_num_errors(wpc);
    if (nch) *nch = ch;
    free(tmp);
    wvo_close(wpc);
    return rv < 0 ? rv : total;
}

int wvo_format_samples(const int32_t *src, int64_t samcnt, int bps, uint8_t *pcm, int64_t pcm_len, int offset,
                       int dsd) /* WavPackUtils.cs:288-341 */
{
    int64_t counter = offset, c2 = 0;
    int64_t len = samcnt * bps;
    if (pcm == NULL || pcm_len < len + offset) return 0;
    switch (bps) {
    case 1:
        if (dsd)
            while (samcnt-- > 0) pcm[counter++] = (uint8_t)src[c2++];
        else
            while (samcnt-- > 0) pcm[counter++] = (uint8_t)(0x00FF & (src[c2++] + 128));
        break;
    case 2:
        while (samcnt-- > 0) {
            int t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
        }
        break;
    case 3:
        while (samcnt-- > 0) {
            int t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
            pcm[counter++] = (uint8_t)(t >> 16);
        }
        break;
    case 4:
        while (samcnt-- > 0) {
            int t = src[c2++];
            pcm[counter++] = (uint8_t)t;
            pcm[counter++] = (uint8_t)(t >> 8);
            pcm[counter++] = (uint8_t)(t >> 16);
            pcm[counter++] = (uint8_t)(t >> 24); /* SupportClass.URShift low byte == t >> 24 */
        }
        break;
    }
    return 1;
}

/* getters: WavPackUtils.cs:346-499 */
int64_t wvo_get_num_samples(wvo_ctx *c, int native) { return native && c->dsd_multiplier > 0 ? c->total_samples * 8 : c->total_samples; }
int64_t wvo_get_sample_index(wvo_ctx *c) { return c->stream.sample_index; }
int64_t wvo_get_num_errors(wvo_ctx *c) { return c->crc_errors; }
int wvo_lossy(wvo_ctx *c) { return c->lossy_blocks || (c->config.flags & CONFIG_HYBRID_FLAG) != 0; }
int64_t wvo_get_sample_rate(wvo_ctx *c)
{
    if (c->config.sample_rate != 0)
        return c->dsd_multiplier > 0 ? (int64_t)c->dsd_multiplier * c->config.sample_rate * 8 : c->config.sample_rate;
    return 44100;
}
int wvo_get_num_channels(wvo_ctx *c) { return c->config.num_channels != 0 ? c->config.num_channels : 2; }
int wvo_get_bits_per_sample(wvo_ctx *c)
{
    if (c->config.bits_per_sample != 0)
        return c->dsd_multiplier > 0 ? c->config.bits_per_sample / 8 : c->config.bits_per_sample;
    return 16;
}
int wvo_get_bytes_per_sample(wvo_ctx *c) { return c->config.bytes_per_sample != 0 ? c->config.bytes_per_sample : 2; }
int wvo_get_reduced_channels(wvo_ctx *c)
{
    if (c->reduced_channels != 0) return c->reduced_channels;
    if (c->config.num_channels != 0) return c->config.num_channels;
    return 2;
}
int wvo_get_mode(wvo_ctx *c) /* WavPackUtils.cs:133-167 */
{
    int mode = 0;
    if ((c->config.flags & CONFIG_HYBRID_FLAG) != 0)
        mode |= MODE_HYBRID;
    else if ((c->config.flags & CONFIG_LOSSY_MODE) == 0)
        mode |= MODE_LOSSLESS;
    if (c->lossy_blocks) mode &= ~MODE_LOSSLESS;
    if ((c->config.flags & CONFIG_FLOAT_DATA) != 0) mode |= MODE_FLOAT;
    if ((c->config.flags & CONFIG_HIGH_FLAG) != 0) {
        mode |= MODE_HIGH;
        if ((c->config.flags & CONFIG_VERY_HIGH_FLAG) > 0 || (c->stream.wphdr.version < 0x405)) mode |= MODE_VERY_HIGH;
    }
    if ((c->config.flags & CONFIG_FAST_FLAG) != 0) mode |= MODE_FAST;
    if ((c->config.flags & CONFIG_EXTRA_MODE) != 0) mode |= MODE_EXTRA | ((c->config.xmode << 12) & MODE_XMODE);
    if (c->dsd_multiplier > 0) mode |= MODE_DSD;
    return mode;
}
int wvo_get_version(wvo_ctx *c) { return c->stream.wphdr.version; }
int wvo_get_is_float(wvo_ctx *c) { return (c->config.flags & CONFIG_FLOAT_DATA) > 0; }
int wvo_get_is_five(wvo_ctx *c) { return c->five; }
int wvo_get_file_format(wvo_ctx *c) { return c->file_format; }
const char *wvo_get_error_message(wvo_ctx *c) { return c->error_message; }
int wvo_exception(wvo_ctx *c) { return c->exception; }
const uint8_t *wvo_get_header(wvo_ctx *c, int *len) { *len = c->header_len; return c->header; }
const uint8_t *wvo_get_trailer(wvo_ctx *c, int *len) { *len = c->trailer_len; return c->trailer; }
void wvo_free(void *p) { free(p); }

int64_t wvo_decode_file(const uint8_t *file, size_t len, int32_t *out, int64_t out_cap, int chunk,
                        int64_t *crc_errors, int *lossy, int *nch)
{
    wvo_ctx *wpc = wvo_open(file, len, 0);
    if (wpc->error_message && wpc->error_message[0]) {
        wvo_close(wpc);
        return -2;
    }
    int ch = wvo_get_reduced_channels(wpc);
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (size_t)chunk * (size_t)ch);
    int64_t total = 0, got;
    int64_t rv = 0;
    while (1) {
        got = wvo_unpack_samples(wpc, tmp, (int64_t)chunk * ch, chunk);
        if (got < 0) { rv = -3; break; }
        if (got > 0) {
            int64_t n = got * ch;
            if ((total * ch + n) <= out_cap) memcpy(out + total * ch, tmp, sizeof(int32_t) * (size_t)n);
            total += got;
        }
        if (got == 0) break;
    }
    if (crc_errors) *crc_errors = wvo_get_num_errors(wpc);
    if (lossy) *lossy = wvo_lossy(wpc);
    if (nch) *nch = ch;
    free(tmp);
    wvo_close(wpc);
    return rv < 0 ? rv : total;
}

/* ------------------------------------------------------------------ */
/* WvDemo.cs + ChunkHeader/RiffChunkHeader/WaveHeader.cs               */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t *p;
    size_t n, cap;
} obuf;
static void ob_put(obuf *o, const void *d, size_t n)
{
    if (o->n + n > o->cap) {
        o->cap = (o->n + n) * 2 + 64;
        o->p = (uint8_t *)realloc(o->p, o->cap);
    }
    memcpy(o->p + o->n, d, n);
    o->n += n;
}
static void le32(uint8_t *b, uint32_t v) { b[0] = (uint8_t)v; b[1] = (uint8_t)(v >> 8); b[2] = (uint8_t)(v >> 16); b[3] = (uint8_t)(v >> 24); }

int wvo_demo(const uint8_t *file, size_t len, uint8_t **wav, size_t *wav_len) /* WvDemo.cs:15-168 */
{
    obuf o = {0};
    int64_t total_unpacked_samples = 0;
    int rc = 0;
    *wav = NULL;
    *wav_len = 0;
    wvo_ctx *wpc = wvo_open(file, len, 0);
    if (wpc->error_message && wpc->error_message[0]) {
        wvo_close(wpc);
        return 1;
    }
    int num_channels = wvo_get_reduced_channels(wpc);
    int bits = wvo_get_bits_per_sample(wpc);
    int byteps = wvo_get_bytes_per_sample(wpc);
    int block_align = byteps * num_channels;
    int64_t total_samples = wvo_get_num_samples(wpc, 1);
    int64_t sample_rate = wvo_get_sample_rate(wpc);
    int hlen;
    const uint8_t *header = wvo_get_header(wpc, &hlen);
    if (header != NULL && !wvo_get_is_float(wpc))
        ob_put(&o, header, (size_t)hlen);
    else {
        uint8_t h[44];
        uint32_t riff = (uint32_t)(total_samples * block_align + 2 * 8 + 16) + 4;
        memcpy(h, "RIFF", 4); le32(h + 4, riff); memcpy(h + 8, "WAVE", 4);          /* RiffChunkHeader.cs:66-87 */
        memcpy(h + 12, "fmt ", 4); le32(h + 16, 16);                                 /* ChunkHeader.cs:29-45 */
        h[20] = 1; h[21] = 0;                                                        /* WaveHeader.cs:109-142 */
        h[22] = (uint8_t)num_channels; h[23] = (uint8_t)(num_channels >> 8);
        le32(h + 24, (uint32_t)sample_rate);
        le32(h + 28, (uint32_t)(sample_rate * block_align));
        h[32] = (uint8_t)block_align; h[33] = (uint8_t)(block_align >> 8);
        h[34] = (uint8_t)bits; h[35] = (uint8_t)(bits >> 8);
        memcpy(h + 36, "data", 4); le32(h + 40, (uint32_t)(total_samples * block_align));
        ob_put(&o, h, 44);
    }
    int samples_unpack = SAMPLE_BUFFER_SIZE;
    int64_t loop_samples = total_samples / 100 / samples_unpack * samples_unpack;
    int32_t *temp_buffer = (int32_t *)calloc((size_t)samples_unpack * num_channels, sizeof(int32_t));
    int64_t pcm_len = (int64_t)samples_unpack * block_align;
    uint8_t *pcm_buffer = (uint8_t *)calloc((size_t)pcm_len, 1);
    while (1) {
        int64_t su = wvo_unpack_samples(wpc, temp_buffer, (int64_t)samples_unpack * num_channels, samples_unpack);
        if (su < 0) { rc = 1; break; } /* exception -> catch (WvDemo.cs:144-149) */
        total_unpacked_samples += su;
        if (su > 0) {
            if (!wvo_format_samples(temp_buffer, su * num_channels, byteps, pcm_buffer, pcm_len, 0, 0)) break;
            ob_put(&o, pcm_buffer, (size_t)(su * block_align));
        }
        if (loop_samples == 0) { rc = 1; break; } /* `%` by zero: DivideByZeroException (WvDemo.cs:130) */
        if (su == 0) break;
    }
    if (rc == 0) {
        int tlen;
        const uint8_t *trailer = wvo_get_trailer(wpc, &tlen);
        if (trailer != NULL) ob_put(&o, trailer, (size_t)tlen);
        int64_t num_samples = wvo_get_num_samples(wpc, 0);
        if (num_samples != -1 && total_unpacked_samples != num_samples) rc = 1;
        else if (wvo_get_num_errors(wpc) > 0) rc = 1;
    }
    free(temp_buffer);
    free(pcm_buffer);
    wvo_close(wpc);
    *wav = o.p;
    *wav_len = o.n;
    return rc;
}

/* ------------------------------------------------------------------ */
/* known-answer test exports                                           */
/* ------------------------------------------------------------------ */
int wvo_exp2s(int log) { return exp2s(log); }
int wvo_count_bits(int64_t av)
{
    jmp_buf jb, *saved = g_jmp;
    int r;
    g_jmp = &jb;
    if (setjmp(jb)) { g_jmp = saved; return -1; }
    r = count_bits(av);
    g_jmp = saved;
    return r;
}
int wvo_mylog2(int64_t avalue)
{
    jmp_buf jb, *saved = g_jmp;
    int r;
    g_jmp = &jb;
    if (setjmp(jb)) { g_jmp = saved; return -1; }
    r = mylog2(avalue);
    g_jmp = saved;
    return r;
}
int wvo_log2s(int value) { return value < 0 ? -wvo_mylog2(-(int64_t)value) : wvo_mylog2(value); }
int wvo_restore_weight(int8_t w) { return restore_weight(w); }
int64_t wvo_read_code_bytes(const uint8_t *bytes, int len, int64_t maxcode, int *used)
{
    jmp_buf jb, *saved = g_jmp;
    uint8_t *copy = (uint8_t *)malloc((size_t)(len > 0 ? len : 1));
    memcpy(copy, bytes, (size_t)len);
    Bitstream bs = bs_open_read(copy, len, 0, len);
    int64_t code;
    g_jmp = &jb;
    if (setjmp(jb)) { g_jmp = saved; free(copy); *used = -1; return -1; }
    code = read_code(&bs, maxcode);
    g_jmp = saved;
    /* bits consumed = 8 * (bytes fetched) - bits still buffered */
    *used = (bs.ptr + 1) * 8 - bs.bc;
    free(copy);
    return code;
}
