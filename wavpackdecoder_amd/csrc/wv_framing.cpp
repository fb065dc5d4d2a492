// wv_framing.cpp -- host framing for the MI355X WavPack decode path.
// See wv_framing.h.  Every routine names the reference code it restates.
#include "wv_framing.h"

#include <string.h>

#include <memory>
#include <stdexcept>

#include "wv_format.h"

namespace wvg {
using namespace wvf;

namespace {

struct CsException : std::exception {};  // a C# exception escaping to the caller (WvDemo.cs:144)

// ---- reference state that matters to the framing -------------------------
struct Hdr {  // WavpackHeader.cs:15-22
    uint32_t ckSize = 0;
    int16_t version = 0;
    int64_t total_samples = 0, block_index = 0;
    uint32_t block_samples = 0, flags = 0;
    int32_t crc = 0;
    bool error = false;
    int64_t stream_position = 0, average_block_size = 0;
};

struct Pass {  // decorr_pass.cs:24-26 + "does the host know its value"
    int16_t term = 0, delta = 0, wA = 0, wB = 0;
    int32_t sA[8] = {0}, sB[8] = {0};
    bool known_w = true, known_s = true;
};

struct Words {  // words_data.cs
    int32_t med[2][3] = {{0, 0, 0}, {0, 0, 0}};
    int32_t slow[2] = {0, 0};
    int64_t acc[2] = {0, 0}, dlt[2] = {0, 0};
    bool known = true;
    // with !known: the fields a later read_hybrid_profile re-sent
    bool known_slow[2] = {true, true}, known_acc[2] = {true, true}, known_dlt[2] = {true, true};
};

struct BitsRef {  // a Bitstream reference: where its bytes are and whether it is untouched
    bool valid = false;
    int64_t file_off = 0;
    int32_t byte_length = 0;  // bs.end
    int32_t data_len = 0;     // C# data.Length
    bool fresh = false;       // opened in the current unpack_init and not yet read
};

struct DsdState {  // WavpackStream.dsds
    bool ready = false, fresh = false;
    int mode = 0;
    int64_t data_off = 0;  // file offset of data[0]
    int32_t data_len = 0;  // data.Length
    int32_t byteptr = 0;   // after init
    int history_bins = 0;
    std::vector<uint8_t> prob;
    std::vector<uint16_t> summed;
    std::vector<uint8_t> lookup;
    std::vector<int32_t> value_lookup;
    int32_t filt[2][7];
    int rate_i = 0;
    int max_prob = 0;       // mode 1: max_probability
    int32_t prob_ptr = 0;   // mode 1: data index of the probability data
};

struct Reader {  // System.IO.BinaryReader over the file bytes
    const uint8_t *d = nullptr;
    int64_t len = 0, pos = 0;
    int byte() { return pos < len ? d[pos++] : -1; }
    int read(uint8_t *dst, int n) {
        int64_t a = len - pos;
        if (a < 0) a = 0;
        if (n > a) n = (int)a;
        if (n > 0) memcpy(dst, d + pos, (size_t)n);
        pos += n;
        return n;
    }
};

struct Md {  // WavpackMetadata.cs:15-23
    int byte_length = 0;
    const uint8_t *data = nullptr;  // read_buffer, or the file bytes for a large sub-block
    int data_len = 0;
    int64_t data_file_off = 0;  // where data[0] came from
    uint8_t id = 0;
    bool hasdata = false;
    int64_t bytecount = 24;
    uint8_t at(int64_t i) const {
        if (i < 0 || i >= data_len) throw CsException();
        return data[i];
    }
};

int exp2s(int log) {
    if (log == INT32_MIN) throw CsException();  // C# recursion never ends (StackOverflow)
    return exp2s_host(log);
}

class Framer {
  public:
    // WavpackContext fields (WavpackContext.cs:15-35) + WavpackStream
    Reader in;
    uint8_t read_buffer[BITSTREAM_BUFFER_SIZE];
    std::string error_message;
    int64_t total_samples = -1;
    int reduced_channels = 0;
    bool lossy_blocks = false, five = false;
    int file_format = 0;
    uint32_t dsd_multiplier = 0;
    int64_t header_off = -1, header_len = 0, trailer_off = -1, trailer_len = 0;
    // config (WavpackConfig.cs)
    int bits_per_sample = 0, bytes_per_sample = 0, num_channels = 0, float_norm_exp_cfg = 0;
    int64_t cfg_flags = 0, sample_rate = 0, channel_mask = 0;
    uint8_t xmode = 0;
    // stream
    Hdr wphdr;
    BitsRef wvbits, wvcbits, wvxbits;
    bool wvx_fresh = false;
    int wvx_skip_bits = 0;
    int32_t crc_mvx = 0;
    Words w;
    int num_terms = 0;
    Pass passes[16];
    int16_t int32_sent_bits = 0, int32_zeros = 0, int32_ones = 0, int32_dups = 0;
    int16_t float_flags = 0, float_shift = 0, float_max_exp = 0, float_norm_exp = 0;
    uint8_t int32_max_width = 0;
    int64_t sample_index = 0;
    DsdState dsd;
    bool inited_this_block = false;  // unpack_init ran for the current header
    bool decoded_since_init = false; // a block was decoded after the last unpack_init
    // deferred metadata values (wv_meta.h): reads whose values the device
    // computes; until materialize() the host copies of those values are stale
    bool defer = false;
    std::vector<MetaItem> pending;  // file offsets, stream order
    // the .wvc correction file (beyond the reference): its blocks are
    // matched to the main stream's by block_index, walked forward from wvc_pos
    const uint8_t *wvc = nullptr;
    int64_t wvc_len = 0, wvc_pos = 0;
    uint64_t wvc_base = 0;
    bool exact_float = false;  // OPEN_EXACT_FLOAT (beyond the reference)

    Framer() {
        memset(read_buffer, 0, sizeof(read_buffer));
        // `new Bitstream()` (WavpackStream.cs:48): non-null, end == 0
        wvbits.valid = true;
        wvbits.byte_length = 0;
        wvbits.fresh = false;
    }

    // ---- WavPackUtils.cs:600-671
    void read_next_header() {
        uint8_t b[32];
        int64_t bytes_skipped = 0;
        int bleft = 0, counter;
        for (;;) {
            for (int i = 0; i < bleft; i++) b[i] = b[32 - bleft + i];
            counter = 0;
            int cnt = 32 - bleft;
            if (in.read(b + bleft, cnt) != cnt) {
                wphdr.error = true;
                return;
            }
            bleft = 32;
            if (b[0] == 'w' && b[1] == 'v' && b[2] == 'p' && b[3] == 'k' && (b[4] & 1) == 0 && b[6] < 16 &&
                b[7] == 0 && b[9] == 4 && b[8] >= (MIN_STREAM_VERS & 0xff) && b[8] <= (MAX_STREAM_VERS & 0xff)) {
                wphdr.ckSize = (uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24);
                wphdr.version = (int16_t)((b[9] << 8) | b[8]);
                wphdr.total_samples = (int64_t)(((uint64_t)b[11] << 32) | ((uint64_t)b[15] << 24) |
                                                ((uint64_t)b[14] << 16) | ((uint64_t)b[13] << 8) | b[12]);
                wphdr.block_index = (int64_t)(((uint64_t)b[10] << 32) | ((uint64_t)b[19] << 24) |
                                              ((uint64_t)b[18] << 16) | ((uint64_t)b[17] << 8) | b[16]);
                wphdr.block_samples = (uint32_t)b[20] | ((uint32_t)b[21] << 8) | ((uint32_t)b[22] << 16) | ((uint32_t)b[23] << 24);
                wphdr.flags = (uint32_t)b[24] | ((uint32_t)b[25] << 8) | ((uint32_t)b[26] << 16) | ((uint32_t)b[27] << 24);
                wphdr.crc = (int32_t)((uint32_t)b[28] | ((uint32_t)b[29] << 8) | ((uint32_t)b[30] << 16) | ((uint32_t)b[31] << 24));
                wphdr.error = false;
                wphdr.stream_position = in.pos - bleft;
                wphdr.average_block_size =
                    wphdr.average_block_size == 0 ? wphdr.ckSize : (wphdr.average_block_size + wphdr.ckSize) / 2;
                inited_this_block = false;
                return;
            }
            counter++;
            bleft--;
            while (bleft > 0 && b[counter] != 'w') {
                counter++;
                bleft--;
            }
            bytes_skipped += counter;
            if (bytes_skipped > 1048576LL) {
                wphdr.error = true;
                return;
            }
        }
    }

    // ---- MetadataUtils.cs:15-109
    bool read_metadata_buff(Md &m) {
        if (m.bytecount >= wphdr.ckSize) return false;
        int a = in.byte();
        if (a < 0) return false;
        m.id = (uint8_t)a;
        int t = in.byte();
        if (t < 0) return false;
        m.bytecount += 2;
        m.byte_length = t << 1;
        if (m.id & ID_LARGE) {
            m.id &= (uint8_t)~ID_LARGE;
            if ((t = in.byte()) < 0) return false;
            m.byte_length += t << 9;
            if ((t = in.byte()) < 0) return false;
            m.byte_length += t << 17;
            m.bytecount += 2;
        }
        int bytes_to_read = m.byte_length;
        if (m.id & ID_ODD_SIZE) {
            m.id &= (uint8_t)~ID_ODD_SIZE;
            m.byte_length--;
        }
        if (m.byte_length == 0) {
            m.hasdata = false;
            return true;
        }
        m.bytecount += bytes_to_read;
        if (bytes_to_read > 0) {
            m.data_file_off = in.pos;
            if (bytes_to_read > BITSTREAM_BUFFER_SIZE) {
                // C# allocates a fresh array and fills it from the stream; a short read
                // fails the block, so the view of the file bytes is the same data
                if (in.len - in.pos < bytes_to_read) {
                    in.pos = in.len;
                    m.hasdata = false;
                    return false;
                }
                m.data = in.d + in.pos;
                m.data_len = bytes_to_read;
                in.pos += bytes_to_read;
            } else {
                m.data = read_buffer;
                m.data_len = BITSTREAM_BUFFER_SIZE;
                if (in.read(read_buffer, bytes_to_read) != bytes_to_read) {
                    m.hasdata = false;
                    return false;
                }
            }
            m.hasdata = true;
        }
        return true;
    }

    // WavpackMetadata.copy_data (WavpackMetadata.cs:25-36): returns C# data.Length after the copy
    bool copy_data(Md &m, int &len) {
        if (!m.hasdata || m.byte_length <= 0) return false;
        len = (m.data_len != BITSTREAM_BUFFER_SIZE) ? m.data_len : m.byte_length;
        return true;
    }

    // ---- deferred values ---------------------------------------------------
    struct Vals {  // meta_apply's view of the host state
        int32_t median[2][3], slow_level[2];
        int64_t bitrate_acc[2], bitrate_delta[2];
        int16_t weight_A[16], weight_B[16];
        int32_t samples_A[16][8], samples_B[16][8];
    };
    // run the pending reads on the host state (before a reader that needs it)
    void materialize() {
        if (pending.empty()) return;
        Vals v;
        memcpy(v.median, w.med, sizeof(v.median));
        memcpy(v.slow_level, w.slow, sizeof(v.slow_level));
        memcpy(v.bitrate_acc, w.acc, sizeof(v.bitrate_acc));
        memcpy(v.bitrate_delta, w.dlt, sizeof(v.bitrate_delta));
        for (int i = 0; i < 16; i++) {
            v.weight_A[i] = passes[i].wA;
            v.weight_B[i] = passes[i].wB;
            memcpy(v.samples_A[i], passes[i].sA, sizeof(v.samples_A[i]));
            memcpy(v.samples_B[i], passes[i].sB, sizeof(v.samples_B[i]));
        }
        for (const MetaItem &it : pending) meta_apply(v, it, in.d);
        memcpy(w.med, v.median, sizeof(v.median));
        memcpy(w.slow, v.slow_level, sizeof(v.slow_level));
        memcpy(w.acc, v.bitrate_acc, sizeof(v.bitrate_acc));
        memcpy(w.dlt, v.bitrate_delta, sizeof(v.bitrate_delta));
        for (int i = 0; i < 16; i++) {
            passes[i].wA = v.weight_A[i];
            passes[i].wB = v.weight_B[i];
            memcpy(passes[i].sA, v.samples_A[i], sizeof(v.samples_A[i]));
            memcpy(passes[i].sB, v.samples_B[i], sizeof(v.samples_B[i]));
        }
        pending.clear();
    }
    // an item whose fields a later read overwrites completely is dropped
    void drop_pending(uint32_t k0, uint32_t k1) {
        size_t o = 0;
        for (size_t i = 0; i < pending.size(); i++)
            if (pending[i].kind != k0 && pending[i].kind != k1) pending[o++] = pending[i];
        pending.resize(o);
    }
    void defer_read(const Md &m, uint32_t kind, int32_t arg, int32_t counter0 = 0) {
        MetaItem it;
        it.off = (uint64_t)m.data_file_off;
        it.kind = kind;
        it.len = (uint32_t)m.byte_length;
        it.num_terms = num_terms;
        it.arg = arg;
        it.counter0 = counter0;
        it.mono = (wphdr.flags & MONO_DATA) ? 1u : 0u;
        pending.push_back(it);
        if (pending.size() > 12) materialize();  // an odd stream: keep the device jobs short
    }

    // ---- readers ------------------------------------------------------------
    bool read_decorr_terms(Md &m) {  // UnpackUtils.cs:156-187
        int termcnt = m.byte_length;
        if (termcnt > MAX_NTERMS) return false;
        Pass tmp[16];
        for (int dc = termcnt - 1, c = 0; dc >= 0; dc--, c++) {
            int b = m.at(c);
            tmp[dc].term = (int16_t)((b & 0x1f) - 5);
            tmp[dc].delta = (int16_t)((b >> 5) & 7);
            if (tmp[dc].term < -3 || (tmp[dc].term > MAX_TERM && tmp[dc].term < 17) || tmp[dc].term > 18) return false;
        }
        for (int i = 0; i < 16; i++) passes[i] = tmp[i];
        num_terms = termcnt;
        drop_pending(META_WEIGHTS, META_SAMPLES);  // every pass was just reset
        return true;
    }
    bool read_decorr_weights(Md &m) {  // UnpackUtils.cs:196-239
        int termcnt = m.byte_length;
        bool mono = (wphdr.flags & MONO_DATA) != 0;
        if (!mono) termcnt /= 2;
        if (termcnt > num_terms) return false;
        if (defer) {  // reads stay inside the sub-block and cannot fail
            for (int k = 0; k < termcnt; k++) passes[num_terms - 1 - k].known_w = true;
            if (termcnt > 0) defer_read(m, META_WEIGHTS, termcnt);
            return true;
        }
        materialize();
        int16_t wa = 0, wb = 0;
        int counter = 0, it = num_terms;
        while (termcnt > 0) {
            int idx = it - 1;
            if (idx < 0 || idx >= 16) throw CsException();
            wa = (int16_t)restore_weight((int8_t)m.at(counter++));
            passes[idx].wA = wa;
            if (!mono) wb = (int16_t)restore_weight((int8_t)m.at(counter++));
            passes[idx].wB = wb;
            passes[idx].known_w = true;
            it--;
            termcnt--;
        }
        return true;
    }
    bool read_decorr_samples(Md &m) {  // UnpackUtils.cs:250-360 (quirk B-7 kept)
        if (defer) {
            // deferred when every iteration reads inside the sub-block and the
            // passes do not run out (else the C# reads stale buffer bytes or throws)
            const bool mono = (wphdr.flags & MONO_DATA) != 0;
            const int q = num_terms > 0 ? passes[num_terms - 1].term : 0;
            const int c0 = (wphdr.version == 0x402 && (wphdr.flags & HYBRID_FLAG)) ? (mono ? 2 : 4) : 0;
            const int step = meta_samples_step(q, mono), span = m.byte_length - c0;
            bool ok = span <= 0 || (step > 0 && span % step == 0 && span / step <= num_terms);
            if (ok) {
                for (int i = 0; i < num_terms; i++) passes[i].known_s = true;
                if (num_terms > 0) defer_read(m, META_SAMPLES, q, c0);
                return true;
            }
        }
        materialize();
        int16_t term = 0;
        int32_t tA[8] = {0}, tB[8] = {0};
        int idx = 0;
        for (int t = num_terms; t > 0; t--) {
            if (idx >= 16) throw CsException();
            term = passes[idx].term;
            memset(passes[idx].sA, 0, sizeof(passes[idx].sA));
            memset(passes[idx].sB, 0, sizeof(passes[idx].sB));
            passes[idx].known_s = true;
            idx++;
        }
        int counter = 0;
        bool mono = (wphdr.flags & MONO_DATA) != 0;
        if (wphdr.version == 0x402 && (wphdr.flags & HYBRID_FLAG)) counter += mono ? 2 : 4;
        idx--;
        auto rd = [&](int o) { return exp2s((int16_t)(m.at(o) + (m.at(o + 1) << 8))); };
        while (counter < m.byte_length) {
            if (term > MAX_TERM) {
                tA[0] = rd(counter);
                tA[1] = rd(counter + 2);
                counter += 4;
                if (!mono) {
                    tB[0] = rd(counter);
                    tB[1] = rd(counter + 2);
                    counter += 4;
                }
            } else if (term < 0) {
                tA[0] = rd(counter);
                tB[0] = rd(counter + 2);
                counter += 4;
            } else {
                for (int mm = 0, cnt = term; cnt > 0; mm++, cnt--) {
                    tA[mm] = rd(counter);
                    counter += 2;
                    if (!mono) {
                        tB[mm] = rd(counter);
                        counter += 2;
                    }
                }
            }
            if (idx < 0 || idx >= 16) throw CsException();
            memcpy(passes[idx].sA, tA, sizeof(tA));
            memcpy(passes[idx].sB, tB, sizeof(tB));
            passes[idx].known_s = true;
            idx--;
        }
        return true;
    }
    bool read_entropy_vars(Md &m) {  // WordsUtils.cs:75-116
        if (defer && ((wphdr.flags & MONO_DATA) ? m.byte_length >= 6 : m.byte_length == 12)) {
            drop_pending(META_ENTROPY, META_HYBRID);  // `w = new words_data()`
            w.known = true;
            defer_read(m, META_ENTROPY, 0);
            return true;
        }
        materialize();
        int b[12];
        for (int i = 0; i < 6; i++) b[i] = m.at(i);
        bool mono = (wphdr.flags & MONO_DATA) != 0;
        if (m.byte_length != 12 && !mono) return false;
        Words nw;
        nw.med[0][0] = exp2s(b[0] + (b[1] << 8));
        nw.med[0][1] = exp2s(b[2] + (b[3] << 8));
        nw.med[0][2] = exp2s(b[4] + (b[5] << 8));
        if (!mono) {
            for (int i = 6; i < 12; i++) b[i] = m.at(i);
            nw.med[1][0] = exp2s(b[6] + (b[7] << 8));
            nw.med[1][1] = exp2s(b[8] + (b[9] << 8));
            nw.med[1][2] = exp2s(b[10] + (b[11] << 8));
        }
        nw.known = true;
        w = nw;
        return true;
    }
    // the fields read_hybrid_profile writes (WordsUtils.cs:132-181)
    void hybrid_known(int byte_length) {
        const bool mono = (wphdr.flags & MONO_DATA) != 0;
        const int w2 = mono ? 2 : 4;
        int bc = w2;
        if (wphdr.flags & HYBRID_BITRATE) {
            w.known_slow[0] = true;
            if (!mono) w.known_slow[1] = true;
            bc += w2;
        }
        w.known_acc[0] = true;
        if (!mono) w.known_acc[1] = true;
        // bitrate_delta: read per channel when bytes remain (WordsUtils.cs:164-178:
        // a mono block writes only channel 0, channel 1 keeps its old value),
        // otherwise both channels are zeroed (:183-184) -- so both become known
        if (bc < byte_length) {
            w.known_dlt[0] = true;
            if (!mono) w.known_dlt[1] = true;
        } else {
            w.known_dlt[0] = w.known_dlt[1] = true;
        }
    }
    bool read_hybrid_profile(Md &m) {  // WordsUtils.cs:124-187
        bool mono = (wphdr.flags & MONO_DATA) != 0;
        hybrid_known(m.byte_length);
        if (defer) {  // deferred when it reads exactly the sub-block (no stale bytes, no failure)
            const int w2 = mono ? 2 : 4;
            int need = ((wphdr.flags & HYBRID_BITRATE) ? w2 : 0) + w2;
            if (need < m.byte_length) need += w2;
            if (need == m.byte_length) {
                defer_read(m, META_HYBRID, (int32_t)wphdr.flags);
                return true;
            }
        }
        materialize();
        int bc = 0;
        auto u16 = [&](int o) { return m.at(o) + (m.at(o + 1) << 8); };
        if (wphdr.flags & HYBRID_BITRATE) {
            w.slow[0] = exp2s(u16(bc));
            bc += 2;
            if (!mono) {
                w.slow[1] = exp2s(u16(bc));
                bc += 2;
            }
        }
        w.acc[0] = (int64_t)shl32(u16(bc), 16);
        bc += 2;
        if (!mono) {
            w.acc[1] = (int64_t)shl32(u16(bc), 16);
            bc += 2;
        }
        if (bc < m.byte_length) {
            w.dlt[0] = exp2s((int16_t)u16(bc));
            bc += 2;
            if (!mono) {
                w.dlt[1] = exp2s((int16_t)u16(bc));
                bc += 2;
            }
            if (bc < m.byte_length) return false;
        } else
            w.dlt[0] = w.dlt[1] = 0;
        return true;
    }
    bool init_bits(Md &m, BitsRef &br, int start) {
        int len;
        if (!copy_data(m, len)) return false;
        br.valid = true;
        br.file_off = m.data_file_off + start;
        br.byte_length = m.byte_length;
        br.data_len = len;
        br.fresh = true;
        return true;
    }
    bool init_wvx(Md &m) {  // UnpackUtils.cs:115-147
        int len;
        if (m.byte_length <= 4 || (m.byte_length & 1) || !copy_data(m, len)) return false;
        crc_mvx = (int32_t)((uint32_t)m.at(0) | ((uint32_t)m.at(1) << 8) | ((uint32_t)m.at(2) << 16) |
                            ((uint32_t)m.at(3) << 24));
        wvxbits.valid = true;
        wvxbits.file_off = m.data_file_off + 4;
        wvxbits.byte_length = m.byte_length;
        wvxbits.data_len = len;
        wvxbits.fresh = true;
        wvx_skip_bits = 0;
        if (m.id == ID_WVX_NEW_BITSTREAM) {
            // getbits(5) from the fresh stream: the first byte's low bits (and the second's)
            uint32_t v = (uint32_t)m.at(4) | ((uint32_t)(len > 5 ? m.at(5) : 0) << 8);
            if (wphdr.flags & FLOAT_DATA) {
                wvx_skip_bits = 10;
            } else {
                int32_max_width = (uint8_t)(v & 0x1f);
                wvx_skip_bits = 5;
            }
        }
        return true;
    }
    bool read_int32_info(Md &m) {  // UnpackUtils.cs:367-382
        if (m.byte_length != 4) return false;
        int32_sent_bits = m.at(0);
        int32_zeros = m.at(1);
        int32_ones = m.at(2);
        int32_dups = m.at(3);
        return true;
    }
    bool read_float_info(Md &m) {  // FloatUtils.cs:15-30
        if (m.byte_length != 4) return false;
        float_flags = m.at(0);
        float_shift = m.at(1);
        float_max_exp = m.at(2);
        float_norm_exp = m.at(3);
        return true;
    }
    bool read_channel_info(Md &m) {  // UnpackUtils.cs:389-410
        int bytecnt = m.byte_length, shift = 0, counter = 0;
        if (bytecnt == 0 || bytecnt > 5) return false;
        num_channels = m.at(counter++);
        int64_t mask = 0;
        while (bytecnt >= 0) {
            mask |= (int64_t)shl32(m.at(counter++), shift);
            shift += 8;
            bytecnt--;
        }
        channel_mask = mask;
        return true;
    }
    bool read_config_info(Md &m) {  // UnpackUtils.cs:432-455
        int bytecnt = m.byte_length, counter = 0;
        if (bytecnt >= 3) {
            cfg_flags &= 0xff;
            cfg_flags |= (int64_t)shl32(m.at(counter++), 8);
            cfg_flags |= (int64_t)shl32(m.at(counter++), 16);
            cfg_flags |= (int64_t)shl32(m.at(counter++), 24);
        }
        if (bytecnt >= 4 && (cfg_flags & CONFIG_EXTRA_MODE)) {
            xmode = m.at(counter++);
            bytecnt--;
        }
        if (bytecnt >= 5) five = true;
        return true;
    }
    bool read_sample_rate(Md &m) {  // UnpackUtils.cs:459-473
        if (m.byte_length == 3) {
            sample_rate = m.at(0);
            sample_rate |= (int64_t)shl32(m.at(1), 8);
            sample_rate |= (int64_t)shl32(m.at(2), 16);
        }
        return true;
    }
    void read_hdr_trailer(Md &m, bool trailer) {  // UnpackUtils.cs:475-491
        if (m.byte_length < 0 || m.byte_length > m.data_len) throw CsException();
        if (trailer) {
            trailer_off = m.data_file_off;
            trailer_len = m.byte_length;
        } else {
            header_off = m.data_file_off;
            header_len = m.byte_length;
        }
    }

    // ---- DSD (DsdUtils.cs)
    bool init_dsd_block(Md &m) {  // :17-54
        if (m.byte_length < 2 || m.at(0) > 31) return false;
        int len;
        if (!copy_data(m, len)) return false;
        DsdState d;
        d.data_off = m.data_file_off;
        d.data_len = len;
        const uint8_t *data = m.data;
        d.byteptr = 0;
        dsd_multiplier = 1u << (data[d.byteptr++] & 31);
        d.mode = data[d.byteptr++];
        d.fresh = true;
        bool ok = false;
        if (d.mode == 0) {
            ok = (int64_t)(d.data_len - d.byteptr) ==
                 (int64_t)wphdr.block_samples * ((wphdr.flags & MONO_DATA) ? 1 : 2);
            d.ready = ok;
        } else if (d.mode == 1)
            ok = init_fast(d, data);
        else if (d.mode == 3)
            ok = init_high(d, data);
        dsd = std::move(d);
        return ok;
    }
    bool init_fast(DsdState &d, const uint8_t *data) {  // :149-242
        if (d.byteptr == d.data_len) return false;
        int history_bits = data[d.byteptr++];
        if (d.byteptr == d.data_len || history_bits > 5) return false;
        d.history_bins = 1 << history_bits;
        const int bins = d.history_bins;
        d.lookup.assign((size_t)bins * 1280, 0);
        d.value_lookup.assign((size_t)bins, 0);
        d.summed.assign((size_t)bins * 256, 0);
        d.prob.assign((size_t)bins * 256, 0);
        int max_probability = data[d.byteptr++];
        d.max_prob = max_probability;
        d.prob_ptr = d.byteptr;
        if (max_probability < 0xFF) {
            size_t outptr = 0, outend = d.prob.size();
            while (outptr < outend && d.byteptr < d.data_len) {
                int code = data[d.byteptr++];
                if (code > max_probability) {
                    int z = code - max_probability;
                    while (outptr < outend && z-- > 0) d.prob[outptr++] = 0;
                } else if (code != 0)
                    d.prob[outptr++] = (uint8_t)code;
                else
                    break;
            }
            if (outptr < outend || (d.byteptr < d.data_len && data[d.byteptr++] > 0)) return false;
        } else if ((size_t)(d.data_len - d.byteptr) > d.prob.size()) {
            memcpy(d.prob.data(), data + d.byteptr, d.prob.size());
            d.byteptr += (int32_t)d.prob.size();
        } else
            return false;
        int total = 0, lb = 0;
        for (int bi = 0; bi < bins; bi++) {
            uint16_t sum = 0;
            for (int i = 0; i < 256; i++) d.summed[(size_t)bi * 256 + i] = sum = (uint16_t)(sum + d.prob[(size_t)bi * 256 + i]);
            if (sum) {
                if ((total += sum) > bins * 1280) return false;
                d.value_lookup[(size_t)bi] = lb;
                for (int i = 0; i < 256; i++)
                    for (int c = d.prob[(size_t)bi * 256 + i]; c > 0; c--) d.lookup[(size_t)lb++] = (uint8_t)i;
            }
        }
        if (d.data_len - d.byteptr < 4 || total > bins * 1280) return false;
        d.ready = true;
        return true;
    }
    bool init_high(DsdState &d, const uint8_t *data) {  // :343-389
        bool mono = (wphdr.flags & MONO_DATA) != 0;
        if (d.data_len - d.byteptr < (mono ? 13 : 20)) return false;
        d.rate_i = data[d.byteptr++];
        int rate_s = data[d.byteptr++];
        if (rate_s != 20) return false;
        // init_ptable (:321-341) runs on the device from rate_i (dsd_ptable_init)
        memset(d.filt, 0, sizeof(d.filt));
        for (int ch = 0; ch < (mono ? 1 : 2); ch++) {
            for (int k = 0; k < 5; k++) d.filt[ch][k] = data[d.byteptr++] << 12;
            int f = data[d.byteptr++];
            f |= data[d.byteptr++] << 8;
            d.filt[ch][5] = (int32_t)((uint32_t)f << 16) >> 16;
        }
        d.ready = true;
        return true;
    }

    // ---- MetadataUtils.process_metadata (:111-192)
    bool process_metadata(Md &m) {
        switch (m.id) {
        case ID_DUMMY: return true;
        case ID_DECORR_TERMS: return read_decorr_terms(m);
        case ID_DECORR_WEIGHTS: return read_decorr_weights(m);
        case ID_DECORR_SAMPLES: return read_decorr_samples(m);
        case ID_ENTROPY_VARS: return read_entropy_vars(m);
        case ID_HYBRID_PROFILE: return read_hybrid_profile(m);
        case ID_SHAPING_WEIGHTS: return true;
        case ID_FLOAT_INFO: return read_float_info(m);
        case ID_INT32_INFO: return read_int32_info(m);
        case ID_CHANNEL_INFO: return read_channel_info(m);
        case ID_CONFIG_BLOCK: return read_config_info(m);
        case ID_SAMPLE_RATE: return read_sample_rate(m);
        case ID_WV_BITSTREAM: return init_bits(m, wvbits, 0);
        case ID_WVC_BITSTREAM:
            if (m.byte_length & 1) return false;
            return init_bits(m, wvcbits, 0);
        case ID_WVX_BITSTREAM:
        case ID_WVX_NEW_BITSTREAM: return init_wvx(m);
        case ID_DSD_BLOCK: return init_dsd_block(m);
        case ID_NEW_CONFIG_BLOCK:
            five = true;
            if (m.byte_length >= 1) file_format = m.at(0);
            return true;
        case ID_RIFF_HEADER:
        case ID_ALT_HEADER: read_hdr_trailer(m, false); return true;
        case ID_RIFF_TRAILER:
        case ID_ALT_TRAILER: read_hdr_trailer(m, true); return true;
        case ID_ALT_EXTENSION:
            if (m.byte_length < 0 || m.byte_length > m.data_len) throw CsException();
            return true;
        case ID_BLOCK_CHECKSUM: five = true; return true;
        default: return (m.id & ID_OPTIONAL_DATA) != 0;
        }
    }

    // ---- UnpackUtils.unpack_init (:24-68)
    bool unpack_init() {
        Md m;
        if (wphdr.block_samples > 0 && wphdr.block_index != 0xFFFFFFFFLL) sample_index = wphdr.block_index;
        inited_this_block = true;
        decoded_since_init = false;
        // anything the previous decode adapted is now unknown unless re-sent
        wvbits.fresh = false;
        wvxbits.fresh = false;
        dsd.fresh = false;
        while (read_metadata_buff(m)) {
            if (!process_metadata(m)) {
                error_message = "invalid metadata id " + std::to_string(m.id);
                return false;
            }
        }
        if (m.bytecount != wphdr.ckSize) {
            error_message = "invalid reading WavPack metadata block";
            return false;
        }
        bool bad = (wphdr.block_samples != 0 && (wphdr.flags & DSD_FLAG)) ? !dsd.ready
                                                                          : (!wvbits.valid || wvbits.byte_length == 0);
        if (bad) {
            error_message = "invalid WavPack file";
            return false;
        }
        if (wphdr.block_samples != 0) {
            if ((wphdr.flags & INT32_DATA) && int32_sent_bits != 0 && !wvxbits.valid) lossy_blocks = true;
            if ((wphdr.flags & FLOAT_DATA) &&
                (float_flags & (FLOAT_EXCEPTIONS | FLOAT_ZEROS_SENT | FLOAT_SHIFT_SENT | FLOAT_SHIFT_SAME)))
                lossy_blocks = true;
        }
        return true;
    }

    // state snapshot for one block about to be decoded
    BlockDesc snapshot(uint64_t blob_base, FramingOutput &out) {
        BlockDesc d;
        memset(&d, 0, sizeof(d));
        d.flags = wphdr.flags;
        d.block_samples = wphdr.block_samples;
        d.crc = wphdr.crc;
        uint32_t status = 0;
        const uint32_t flags = wphdr.flags;
        int mag = (int)((flags & MAG_MASK) >> MAG_LSB);
        int32_t ml = (int32_t)((int64_t)(1LL << mag) + 2);
        if (flags & HYBRID_FLAG) ml = mul32(ml, 2);
        d.mute_limit = ml;
        d.shift = (int32_t)((flags & SHIFT_MASK) >> SHIFT_LSB);
        d.float_shift = float_max_exp - float_norm_exp + float_shift;
        d.int32_sent_bits = int32_sent_bits;
        d.int32_zeros = int32_zeros;
        d.int32_ones = int32_ones;
        d.int32_dups = int32_dups;
        d.int32_max_width = int32_max_width;
        // a header whose block was not unpack_init'ed decodes with the stream state
        // left from earlier metadata (sticky state, B-8): known while that state is
        // unconsumed (the fresh/known flags below); once a decode consumed it, the
        // block inherits it from that decode (d.inherit, chained in frame_file)
        uint32_t inh = 0, inhp = 0;
        if (!inited_this_block && decoded_since_init) inh |= INH_NOINIT;
        if (flags & DSD_FLAG) {
            if (!dsd.fresh) inh |= INH_DSD;  // continues a consumed DSD state (chained, frame_file)
            d.kind = dsd.mode == 0 ? KIND_DSD_RAW : dsd.mode == 1 ? KIND_DSD_FAST : KIND_DSD_HIGH;
            d.bits_off = blob_base + (uint64_t)dsd.data_off + (uint64_t)dsd.byteptr;
            d.dsd_data_len = (uint32_t)(dsd.data_len - dsd.byteptr);
            d.dsd_history_bins = dsd.history_bins;
            d.dsd_rate_i = dsd.rate_i;
            if (dsd.mode == 1) {
                // table area: prob[bins*256] u8 | summed[bins*256] u16 | lookup[bins*1280] u8 | value_lookup[bins] i32
                size_t off = (out.tables.size() + 15) & ~(size_t)15;
                size_t bins = (size_t)dsd.history_bins;
                out.tables.resize(off + bins * 256 + bins * 512 + bins * 1280 + bins * 4 + 16, 0);
                uint8_t *t = out.tables.data() + off;
                memcpy(t, dsd.prob.data(), bins * 256);
                memcpy(t + bins * 256, dsd.summed.data(), bins * 512);
                memcpy(t + bins * 768, dsd.lookup.data(), bins * 1280);
                memcpy(t + bins * 2048, dsd.value_lookup.data(), bins * 4);
                d.dsd_table_off = off;
                d.dsd_max_prob = dsd.max_prob;
                d.dsd_prob_off = blob_base + (uint64_t)dsd.data_off + (uint64_t)dsd.prob_ptr;
            } else if (dsd.mode == 3) {  // the kernel builds the ptable from dsd_rate_i (dsd_ptable_init)
                memcpy(d.dsd_filters, dsd.filt, sizeof(d.dsd_filters));
            }
        } else {
            d.kind = KIND_PCM;
            if (!wvbits.fresh) inh |= INH_BITS;  // continues a consumed bitstream
            d.bits_off = blob_base + (uint64_t)wvbits.file_off;
            d.bits_len = (uint32_t)wvbits.byte_length;
            if (wvxbits.valid) {
                d.wvx_state = 1 | (wvx_skip_bits << 1);
                d.crc_mvx = crc_mvx;
                d.wvx_off = blob_base + (uint64_t)wvxbits.file_off;
                d.wvx_len = (uint32_t)(wvxbits.data_len - 4);
                if ((flags & INT32_DATA) && !(flags & FLOAT_DATA)) {
                    // fixup_samples reads it (UnpackUtils.cs:1271-1314)
                    if (!wvxbits.fresh) inh |= INH_WVX;
                    d.wvx_state |= 0x100;
                }
            }
            if (exact_float && (flags & FLOAT_DATA)) {
                // WavPack 4's float_values instead of FloatUtils.cs:32-56 (fixup_xfloat):
                // the block's own classic ID_WVX_BITSTREAM, if any (WavPack opens the
                // stream per block; a NEW-format stream is not decoded)
                d.xfloat = XF_ON | ((uint32_t)float_flags & 0xffu) | (((uint32_t)float_max_exp & 0xffu) << 8) |
                           (((uint32_t)float_shift & 0xffu) << 16);
                if (wvxbits.valid && !wvxbits.fresh) {
                    d.wvx_state = 0;
                    d.wvx_off = 0;
                    d.wvx_len = 0;
                } else if (wvxbits.valid && wvx_skip_bits) {
                    status |= ST_UNSUPPORTED;
                }
            }
            if (!w.known) {
                inh |= INH_ENTROPY;
                for (int c = 0; c < 2; c++) {
                    if (!w.known_slow[c]) inh |= INH_SLOW0 << c;
                    if (!w.known_acc[c]) inh |= INH_ACC0 << c;
                    if (!w.known_dlt[c]) inh |= INH_DLT0 << c;
                }
            }
            memcpy(d.median, w.med, sizeof(d.median));
            memcpy(d.slow_level, w.slow, sizeof(d.slow_level));
            memcpy(d.bitrate_acc, w.acc, sizeof(d.bitrate_acc));
            memcpy(d.bitrate_delta, w.dlt, sizeof(d.bitrate_delta));
            d.num_terms = num_terms;
            for (int i = 0; i < num_terms && i < 16; i++) {
                const Pass &p = passes[i];
                if (!p.known_w) inhp |= 1u << i;
                if (!p.known_s) inhp |= 1u << (16 + i);
                d.term[i] = (int8_t)p.term;
                d.delta[i] = (int8_t)p.delta;
                d.weight_A[i] = p.wA;
                d.weight_B[i] = p.wB;
                memcpy(d.samples_A[i], p.sA, sizeof(p.sA));
                memcpy(d.samples_B[i], p.sB, sizeof(p.sB));
            }
            if (!pending.empty()) {  // the device finishes these values (wv_meta_parse)
                MetaJob j;
                j.desc = (uint32_t)out.descs.size();
                j.first = (uint32_t)out.items.size();
                j.count = (uint32_t)pending.size();
                j.pad_ = 0;
                for (MetaItem it : pending) {
                    it.off += blob_base;
                    out.items.push_back(it);
                }
                out.jobs.push_back(j);
            }
            if (num_terms < 0 || num_terms > 16) status |= ST_UNSUPPORTED;
            // (FALSE_STEREO with MONO_FLAG: 2 ints a frame, the layout rule at the call loop)
            // INT32 sent_bits past 32 with a wvx stream read: getbits past 32 bits
            // (BitsUtils.cs:37-68 on a 32-bit register) -- BitReader::getbits_big
        }
        if (d.kind == KIND_PCM) {
            d.inherit = inh;
            d.inherit_passes = inhp;
            if (!inh && !inhp && !(d.wvx_state & 1)) attach_wvc(d);
        } else {
            // a DSD block continuing the DSD state and / or the crc / mute state of the block
            // decoded before it (chained with it, decode_dsd_chained)
            d.inherit = inh & (INH_DSD | INH_NOINIT);
        }
        if (status & ST_UNSUPPORTED) {
            d.kind = KIND_SKIP;
            d.inherit = d.inherit_passes = 0;
        }
        // the framing reports its verdicts through the same status word
        d.fstatus = status;
        return d;
    }

    // The correction stream of the hybrid block being snapshotted: the .wvc block
    // with the same block_index (its headers back to back, as WavPack writes
    // them), its ID_WVC_BITSTREAM sub-block (even length, UnpackUtils.cs:96-106).
    // d.crc becomes the .wvc header's crc (of the exact output).
    void attach_wvc(BlockDesc &d) {
        if (!wvc || !(wphdr.flags & HYBRID_FLAG) || (wphdr.flags & HYBRID_SHAPE)) return;
        while (wvc_pos + 32 <= wvc_len) {
            const uint8_t *b = wvc + wvc_pos;
            if (!(b[0] == 'w' && b[1] == 'v' && b[2] == 'p' && b[3] == 'k')) return;
            const uint32_t ck = (uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24);
            const int64_t bi = (int64_t)(((uint64_t)b[10] << 32) | ((uint64_t)b[19] << 24) | ((uint64_t)b[18] << 16) |
                                         ((uint64_t)b[17] << 8) | b[16]);
            if (bi > wphdr.block_index) return;
            const int64_t end = wvc_pos + (int64_t)ck + 8;
            if (end > wvc_len) return;
            if (bi == wphdr.block_index) {
                for (int64_t p = wvc_pos + 32; p + 2 <= end;) {
                    uint8_t id = wvc[p];
                    int64_t bl = (int64_t)wvc[p + 1] << 1, hl = 2;
                    if (id & ID_LARGE) {
                        if (p + 4 > end) return;
                        bl += ((int64_t)wvc[p + 2] << 9) + ((int64_t)wvc[p + 3] << 17);
                        hl = 4;
                    }
                    const int64_t real = (id & ID_ODD_SIZE) ? bl - 1 : bl;
                    if ((id & 0x3f) == ID_WVC_BITSTREAM && real > 0 && !(real & 1) && p + hl + bl <= end &&
                        !d.wvc_len) {
                        d.wvc_off = wvc_base + (uint64_t)(p + hl);
                        d.wvc_len = (uint32_t)real;
                        d.crc_lossy = d.crc;
                        d.crc = (int32_t)((uint32_t)b[28] | ((uint32_t)b[29] << 8) | ((uint32_t)b[30] << 16) |
                                          ((uint32_t)b[31] << 24));
                    } else if ((id & 0x3f) == ID_WVX_BITSTREAM && !(id & ID_OPTIONAL_DATA) && (d.xfloat & XF_ON) &&
                               real > 4 && !(real & 1) && p + hl + bl <= end && !(d.wvx_state & 1)) {
                        // exact float of a hybrid float file: its wvx stream sits in the .wvc block
                        const uint8_t *x = wvc + p + hl;
                        d.crc_mvx = (int32_t)((uint32_t)x[0] | ((uint32_t)x[1] << 8) | ((uint32_t)x[2] << 16) |
                                              ((uint32_t)x[3] << 24));
                        d.wvx_off = wvc_base + (uint64_t)(p + hl + 4);
                        d.wvx_len = (uint32_t)(real - 4);
                        d.wvx_state = 1;
                    }
                    p += hl + bl;
                }
                wvc_pos = end;
                return;
            }
            wvc_pos = end;
        }
    }

    // decoding changes the passes, the entropy state and the bitstreams
    void mark_adapted() {
        for (auto &p : passes) p.known_w = p.known_s = false;
        w.known = false;
        for (int c = 0; c < 2; c++) w.known_slow[c] = w.known_acc[c] = w.known_dlt[c] = false;
        decoded_since_init = true;
        wvbits.fresh = false;
        wvxbits.fresh = false;
        dsd.fresh = false;
    }
};

// ---- WavpackOpenFileInput (WavPackUtils.cs:36-120) from the reader's current
// position; false (and the error message) when the reference reports an error
bool open_input(Framer &F, uint32_t open_flags, std::string &err) {
    while (F.wphdr.block_samples == 0) {
        F.read_next_header();
        if (F.wphdr.error) {
            err = "not compatible with this version of WavPack file!";
            return false;
        }
        if (F.wphdr.block_samples > 0 && F.wphdr.total_samples != 0xFFFFFFFFLL) F.total_samples = F.wphdr.total_samples;
        if (!F.unpack_init()) {
            err = F.error_message;
            return false;
        }
    }
    F.cfg_flags = (F.cfg_flags & ~0xffLL) | (F.wphdr.flags & 0xff);
    F.bytes_per_sample = (int)((F.wphdr.flags & BYTES_STORED) + 1);
    F.float_norm_exp_cfg = F.float_norm_exp;
    F.bits_per_sample = (int)(F.bytes_per_sample * 8 - ((F.wphdr.flags & SHIFT_MASK) >> SHIFT_LSB));
    if (F.cfg_flags & FLOAT_DATA) {
        F.bytes_per_sample = 3;
        F.bits_per_sample = 24;
    }
    if (F.sample_rate == 0) {
        static const int64_t rates[15] = {6000,  8000,  9600,  11025, 12000, 16000, 22050, 24000,
                                          32000, 44100, 48000, 64000, 88200, 96000, 192000};
        if (F.wphdr.block_samples == 0 || (F.wphdr.flags & SRATE_MASK) == SRATE_MASK)
            F.sample_rate = 44100;
        else
            F.sample_rate = rates[(F.wphdr.flags & SRATE_MASK) >> SRATE_LSB];
    }
    if (F.num_channels == 0) {
        F.num_channels = (F.wphdr.flags & MONO_FLAG) ? 1 : 2;
        F.channel_mask = 0x5 - F.num_channels;
    }
    if ((open_flags & 0x8) && !(F.wphdr.flags & FINAL_BLOCK)) F.reduced_channels = (F.wphdr.flags & MONO_FLAG) ? 1 : 2;
    if (!(open_flags & 0x8) && F.num_channels > 2) {
        err = "only two channels supported!";
        return false;
    }
    if (F.wphdr.flags & DSD_FLAG) {
        F.bytes_per_sample = 1;
        F.bits_per_sample = 8;
    }
    return true;
}

// `wpc.stream = c.stream` (WavPackUtils.cs:572): the WavpackStream part of the
// state moves; the context part (config, totals, header/trailer, lossy_blocks,
// crc_errors) stays the caller's
void take_stream(Framer &F, const Framer &c) {
    F.wphdr = c.wphdr;
    F.wvbits = c.wvbits;
    F.wvcbits = c.wvcbits;
    F.wvxbits = c.wvxbits;
    F.wvx_fresh = c.wvx_fresh;
    F.wvx_skip_bits = c.wvx_skip_bits;
    F.crc_mvx = c.crc_mvx;
    F.w = c.w;
    F.num_terms = c.num_terms;
    for (int i = 0; i < 16; i++) F.passes[i] = c.passes[i];
    F.int32_sent_bits = c.int32_sent_bits;
    F.int32_zeros = c.int32_zeros;
    F.int32_ones = c.int32_ones;
    F.int32_dups = c.int32_dups;
    F.float_flags = c.float_flags;
    F.float_shift = c.float_shift;
    F.float_max_exp = c.float_max_exp;
    F.float_norm_exp = c.float_norm_exp;
    F.int32_max_width = c.int32_max_width;
    F.sample_index = c.sample_index;
    F.dsd = c.dsd;
    F.inited_this_block = c.inited_this_block;
    F.decoded_since_init = c.decoded_since_init;
    F.pending = c.pending;
}

// SetSample -> seek (WavPackUtils.cs:509-594), restated over the header walk:
// 1 positioned at the block holding `target` (`index` frames into it, still to
// be decoded and discarded), 0 the C# `false` (context untouched), exceptions
// other than IOException escape (CsException)
int seek(Framer &F, int64_t target, int64_t &index) {
    if (target >= F.total_samples) return 0;
    if (target < 0) target = 0;
    int steps = 25;
    const int min = 5;
    while (steps-- > 0) {
        Hdr &h = F.wphdr;
        int64_t seek_pos = h.stream_position;
        if (target <= (int64_t)h.block_samples)
            seek_pos = 0;
        else if (target < h.block_index || target > h.block_index + (int64_t)h.block_samples) {
            int64_t distance = target - h.block_index;
            distance += distance > 0 ? (-1 * (int64_t)h.block_samples + 1) : (-2 * (int64_t)h.block_samples + 1);
            if (h.block_samples == 0) throw CsException();  // DivideByZeroException
            int64_t blocks = distance / (int64_t)h.block_samples;
            if (blocks >= 0 && blocks <= min)
                seek_pos = -1;
            else
                seek_pos += blocks * h.average_block_size;
            if (seek_pos >= F.in.len) seek_pos = -1;
        }
        if (seek_pos != -1) {
            if (seek_pos < 0) return 0;  // Stream.Seek before the start: IOException, caught (:590)
            F.in.pos = seek_pos;
        }
        F.read_next_header();
        if (F.wphdr.error) continue;
        if (steps == 0 || (target >= F.wphdr.block_index && target < F.wphdr.block_index + (int64_t)F.wphdr.block_samples)) {
            index = target - F.wphdr.block_index;
            std::unique_ptr<Framer> c(new Framer());
            c->defer = F.defer;
            c->in = F.in;
            c->in.pos = F.wphdr.stream_position;
            std::string err;
            open_input(*c, 0, err);  // the reference does not look at c's error
            F.in.pos = c->in.pos;    // one BinaryReader
            take_stream(F, *c);
            return 1;
        }
        if (seek_pos == -1) {
            F.in.pos = F.wphdr.stream_position + F.wphdr.ckSize;
            steps--;
        }
    }
    return 0;
}

}  // namespace

void apply_meta_jobs(FramingOutput &out, const uint8_t *blob) {
    for (const MetaJob &j : out.jobs)
        for (uint32_t k = 0; k < j.count; k++) meta_apply(out.descs[j.desc], out.items[j.first + k], blob);
}

int64_t file_out_extent(const FramingOutput &out, const FileInfo &info, uint64_t out_base_ints) {
    int64_t extent = info.out_frames * info.out_nch;
    for (int64_t k = info.first_desc; k < info.first_desc + info.num_desc; k++) {
        const BlockDesc &d = out.descs[(size_t)k];
        const int64_t e = (int64_t)(d.out_off - out_base_ints) + (int64_t)d.nframes * (int64_t)d.out_nch;
        if (e > extent) extent = e;
    }
    return extent;
}

bool dframe_file_info(const DFile &df, const DBlock *r, FileInfo &info) {
    if (!df.regular || df.nblocks == 0) return false;
    // state the host would carry from block to block must be re-sent the same way in
    // every block (INT32/FLOAT info), and the channel count must not change
    const int32_t mask0 = r[0].info_mask;
    bool lossy = false, five = false;
    int32_t file_format = 0, dsd_log2 = -1;
    int64_t hoff = -1, hlen = 0, toff = -1, tlen = 0;
    for (uint32_t k = 0; k < df.nblocks; k++) {
        const DBlock &b = r[k];
        if (!b.regular || b.info_mask != mask0 || (b.num_channels >= 0 && b.num_channels != df.num_channels))
            return false;
        lossy |= b.lossy != 0;
        five |= b.five != 0;
        if (b.file_format >= 0) file_format = b.file_format;
        if (b.dsd_mult_log2 >= 0) dsd_log2 = b.dsd_mult_log2;
        if (b.header_off >= 0) hoff = b.header_off, hlen = b.header_len;
        if (b.trailer_off >= 0) toff = b.trailer_off, tlen = b.trailer_len;
    }
    const uint64_t blob_base = info.blob_base;
    const int64_t first_desc = info.first_desc;
    info = FileInfo();
    info.blob_base = blob_base;
    info.first_desc = first_desc;
    info.num_desc = df.nblocks;
    info.open_ok = 1;
    info.num_channels = df.num_channels;
    info.reduced_channels = 0;
    info.bits_per_sample = df.bits_per_sample;
    info.bytes_per_sample = df.bytes_per_sample;
    info.version = df.version;
    info.mode = df.mode;
    info.is_float = df.is_float;
    info.sample_rate = df.sample_rate;
    info.total_samples = df.total_samples;
    info.config_flags = df.config_flags;
    info.out_nch = df.nch;
    info.out_frames = df.total_samples;
    info.first_call_frames = df.total_samples < (int64_t)df.chunk ? df.total_samples : (int64_t)df.chunk;
    info.sample_index0 = 0;
    info.lossy_blocks = lossy;
    info.is_five = five;
    info.file_format = file_format;
    info.dsd_multiplier = dsd_log2 >= 0 ? 1u << dsd_log2 : 0u;
    info.header_off = hoff;
    info.header_len = hlen;
    info.trailer_off = toff;
    info.trailer_len = tlen;
    return true;
}

int compute_mode(const FileInfo &info) {  // WavPackUtils.cs:133-167 (fields captured at open)
    return info.mode;
}

// Blocks that inherit decode state (d.inherit) join the block decoded before
// them into a chain, back to a block whose state is all in its descriptor; the
// chain's first descriptor records the chain length.  PCM chains continue PCM
// state, DSD chains DSD state; a block whose predecessor is of the other family
// or was skipped stays unsupported (the state it continues was left by a block
// further back: malformed files only).
static void chain_blocks(FramingOutput &out, int64_t first, int64_t count) {
    int64_t head = -1;
    auto family = [](uint32_t kind) { return kind == KIND_PCM ? 0 : (kind == KIND_SKIP ? 2 : 1); };
    for (int64_t k = first; k < first + count; k++) {
        BlockDesc &d = out.descs[(size_t)k];
        if (d.kind == KIND_SKIP || (d.inherit == 0 && d.inherit_passes == 0)) {
            head = d.kind == KIND_SKIP ? -1 : k;
            continue;
        }
        if (head >= 0 && family(out.descs[(size_t)head].kind) != family(d.kind)) head = -1;
        if (head < 0) {
            d.kind = KIND_SKIP;
            d.fstatus |= ST_UNSUPPORTED;
            d.inherit = d.inherit_passes = 0;
            continue;
        }
        BlockDesc &h = out.descs[(size_t)head];
        h.chain_len = h.chain_len ? h.chain_len + 1 : 2;
        d.inherit |= INH_MEMBER;
    }
}

void frame_file(const uint8_t *file, size_t len, uint64_t blob_base, uint64_t out_base_ints, uint32_t open_flags,
                int chunk, FramingOutput &out, FileInfo &info, int64_t seek_to, const uint8_t *wvc, size_t wvc_len,
                uint64_t wvc_base) {
    std::unique_ptr<Framer> FP(new Framer());
    Framer &F = *FP;
    F.defer = out.defer_values;
    F.wvc = wvc;
    F.wvc_len = wvc ? (int64_t)wvc_len : 0;
    F.wvc_base = wvc_base;
    F.exact_float = (open_flags & OPEN_EXACT_FLOAT) != 0;
    F.in.d = file;
    F.in.len = (int64_t)len;
    info = FileInfo();
    info.first_desc = (int64_t)out.descs.size();
    info.blob_base = blob_base;
    const size_t tables0 = out.tables.size();
    try {
        std::string err;
        if (!open_input(F, open_flags, err)) {
            info.error = err;
            return;
        }
    } catch (const CsException &) {
        info.error = "exception";
        info.exception = 1;
        return;
    }
    info.open_ok = 1;
    info.num_channels = F.num_channels;
    info.reduced_channels = F.reduced_channels;
    info.bits_per_sample = F.bits_per_sample;
    info.bytes_per_sample = F.bytes_per_sample;
    info.version = F.wphdr.version;
    info.sample_rate = F.sample_rate;
    info.total_samples = F.total_samples;
    info.config_flags = F.cfg_flags;
    {  // WavpackGetMode at open time
        int mode = 0;
        if (F.cfg_flags & CONFIG_HYBRID_FLAG) mode |= 0x4;
        else if (!(F.cfg_flags & CONFIG_LOSSY_MODE)) mode |= 0x2;
        if (F.lossy_blocks) mode &= ~0x2;
        if (F.cfg_flags & CONFIG_FLOAT_DATA) mode |= 0x8;
        if (F.cfg_flags & CONFIG_HIGH_FLAG) {
            mode |= 0x20;
            if ((F.cfg_flags & CONFIG_VERY_HIGH_FLAG) || F.wphdr.version < 0x405) mode |= 0x400;
        }
        if (F.cfg_flags & CONFIG_FAST_FLAG) mode |= 0x40;
        if (F.cfg_flags & CONFIG_EXTRA_MODE) mode |= 0x80 | ((F.xmode << 12) & 0x7000);
        if (F.dsd_multiplier > 0) mode |= 0x10000;
        info.mode = mode;
    }
    info.is_float = (F.cfg_flags & CONFIG_FLOAT_DATA) != 0;

    const int nch = F.reduced_channels ? F.reduced_channels : F.num_channels;
    info.out_nch = nch;
    int64_t out_frames = 0;
    BlockDesc *cur = nullptr;  // descriptor of the block being decoded
    int64_t cur_idx = -1;
    // ---- SetSample(seek_to) (WavPackUtils.cs:509-594): its discard calls of
    // SAMPLE_BUFFER_SIZE / reduced channels frames decode the start of the block
    int64_t discard = 0;
    const int64_t dchunk = nch > 0 ? 4096 / nch : 4096;
    try {
        if (seek_to >= 0) {
            int64_t index = 0;
            info.seek_result = seek(F, seek_to, index);
            // (when the 25-step search gives up, `index` can exceed the block: the
            // discard then runs on into the next blocks, as in the reference)
            if (info.seek_result == 1 && index > 0) discard = index;
        }
    } catch (const CsException &) {
        info.seek_result = -1;
        info.exception = 1;
        info.num_desc = 0;
        return;
    }
    // ---- the caller's loop (WvDemo.cs:117-135) over WavpackUnpackSamples (WavPackUtils.cs:200-282)
    info.sample_index0 = F.sample_index;
    try {
        for (;;) {
            const bool disc_call = discard > 0;
            if (!disc_call && info.first_call_frames < 0) info.sample_index0 = F.sample_index;
            int64_t samples = disc_call ? (discard < dchunk ? discard : dchunk) : chunk, unpacked = 0;
            int64_t buf_idx = 0;
            while (samples > 0) {
                Hdr &h = F.wphdr;
                if (h.block_samples == 0 || !(h.flags & INITIAL_BLOCK) || F.sample_index >= h.block_index + h.block_samples) {
                    F.read_next_header();
                    if (F.wphdr.error) break;
                    cur_idx = -1;
                    if (F.wphdr.block_samples == 0 || F.sample_index == F.wphdr.block_index) {
                        if (!F.unpack_init()) break;
                    }
                }
                Hdr &hh = F.wphdr;
                if (hh.block_samples == 0 || !(hh.flags & INITIAL_BLOCK) || F.sample_index >= hh.block_index + hh.block_samples)
                    continue;
                if (F.sample_index < hh.block_index) {  // gap: zero fill (the decode writes it, ZeroSeg)
                    int64_t n = hh.block_index - F.sample_index;
                    if (n > samples) n = samples;
                    // (a fill that runs past the caller's buffer throws below, and the call returns nothing)
                    if (!disc_call && n > 0 && buf_idx + n * nch <= (int64_t)chunk * nch)
                        out.zeros.push_back({out_base_ints + (uint64_t)((out_frames + unpacked) * nch), (uint64_t)(n * nch)});
                    F.sample_index += n;
                    unpacked += n;
                    samples -= n;
                    buf_idx += n * nch;
                    if (buf_idx > (int64_t)(disc_call ? 4096 : (int64_t)chunk * nch)) throw CsException();
                    continue;
                }
                int64_t n = hh.block_index + hh.block_samples - F.sample_index;
                if (n > samples) n = samples;
                // one unpack_samples / unpack_dsd_samples call of n frames at buf_idx
                // ints each frame writes: PCM 1 for MONO_FLAG without FALSE_STEREO
                // (UnpackUtils.cs:655-664 copies a false-stereo frame), DSD 1 for MONO_FLAG
                const bool pcm_blk = !(hh.flags & DSD_FLAG);
                const int bch = ((hh.flags & MONO_FLAG) && !(pcm_blk && (hh.flags & FALSE_STEREO))) ? 1 : 2;
                const int64_t buf_len = (int64_t)(disc_call ? 4096 : (int64_t)chunk * nch);
                // a DSD block's unmuted call writes 2 ints a frame on FALSE_STEREO whatever
                // MONO_FLAG says (DsdUtils.cs:119-131), its muted call MONO_FLAG ? 1 : 2
                // (:106-113): both must be the file's width for the block to be decoded here
                const int dsd_wch = (hh.flags & FALSE_STEREO) ? 2 : bch;
                if (!pcm_blk && (bch != nch || dsd_wch != nch)) {
                    // a DSD layout the reference writes inconsistently (and may overrun): not decoded here
                    info.nondet = 1;
                }
                if (cur_idx < 0) {
                    BlockDesc d = F.snapshot(blob_base, out);
                    d.out_off = out_base_ints + (uint64_t)((out_frames + unpacked) * nch);
                    d.first_chunk = (uint32_t)n;
                    d.chunk = (uint32_t)chunk;
                    d.first_bsp = (uint32_t)buf_idx;
                    d.out_nch = (uint32_t)nch;
                    d.call_nch = (F.reduced_channels == 1 || F.num_channels == 1 || (hh.flags & MONO_FLAG)) ? 1 : 2;
                    d.nframes = 0;
                    if (disc_call) {
                        // a block met by the seek's discard calls: its first `rem` frames
                        // go to the dropped temp buffer
                        const int64_t rem = discard - unpacked;
                        d.pre_end = (uint32_t)rem;
                        d.pre_chunk = (uint32_t)dchunk;
                        d.out_off = out_base_ints + (uint64_t)(out_frames * nch) - (uint64_t)(rem * nch);
                    }
                    if (!pcm_blk && (bch != nch || dsd_wch != nch)) {
                        d.kind = KIND_SKIP;
                        d.fstatus |= ST_UNSUPPORTED;
                        d.inherit = d.inherit_passes = 0;
                    }
                    // a PCM block of 1 int a frame in a 2-int file leaves every other slot of
                    // its calls with the caller's stale buffer (decode_pcm_run's store)
                    if (bch != nch && pcm_blk && bch == 1) d.fstatus |= ST_NONDET;
                    if ((hh.flags & DSD_FLAG) && F.dsd.mode == 0 && (hh.flags & FALSE_STEREO)) {
                        // DsdUtils.cs:81 advances bufferStartPos, then :119-131 duplicates
                        // from past it: the reference overruns or emits caller-buffer garbage.
                        d.kind = KIND_SKIP;
                        d.fstatus |= ST_NONDET;
                    }
                    out.descs.push_back(d);
                    cur_idx = (int64_t)out.descs.size() - 1;
                    F.mark_adapted();
                }
                cur = &out.descs[(size_t)cur_idx];
                // the C# array store past the caller's buffer throws in this call, which
                // then returns nothing (the exception escapes WavpackUnpackSamples,
                // WavPackUtils.cs:261): a 2-int PCM block in a 1-int file writes 2n ints
                // from buf_idx; DSD mode 0 + FALSE_STEREO advances bufferStartPos by n
                // (DsdUtils.cs:81) and then expands 2n ints past it (:119-131).  (The
                // frames stay in the descriptor: the device decodes them, nobody reads them.)
                // A DSD FALSE_STEREO block in a 1-int file (declined above) likewise expands 2n
                // ints.  (Known divergence, malformed files only: a call that starts muted
                // zero-fills n ints and returns before the copy, UnpackUtils.cs:527-543 /
                // DsdUtils.cs:104-117, so the reference does not throw there; the framing
                // cannot see the device's mute state and flags the throw.)
                const int wch = pcm_blk ? bch : dsd_wch;  // ints a frame the unmuted call writes
                const bool overrun =
                    (wch == 2 && nch == 1 && buf_idx + 2 * n > buf_len) ||
                    (!pcm_blk && F.dsd.mode == 0 && (hh.flags & FALSE_STEREO) && buf_idx + 3 * n > buf_len);
                cur->nframes += (uint32_t)n;
                if (overrun) throw CsException();
                F.sample_index += n;
                buf_idx += n * nch;
                unpacked += n;
                samples -= n;
                if (F.sample_index == F.total_samples) break;
            }
            if (disc_call) {
                if (unpacked == 0) {  // `index -= 0` forever (WavPackUtils.cs:574-579)
                    info.seek_result = -1;
                    info.exception = 1;
                    break;
                }
                discard -= unpacked;
                continue;
            }
            if (info.first_call_frames < 0) info.first_call_frames = unpacked;
            if (unpacked == 0) break;
            out_frames += unpacked;
            if (unpacked < (int64_t)chunk) info.call_cuts.push_back(out_frames);
            if (info.exception) break;
            // a descriptor whose block stopped exactly at a call boundary stays open:
            // the next call continues it (cur_idx kept)
        }
    } catch (const CsException &) {
        info.exception = 1;
    }
    info.out_frames = out_frames;
    info.lossy_blocks = F.lossy_blocks;
    info.is_five = F.five;
    info.file_format = F.file_format;
    info.dsd_multiplier = F.dsd_multiplier;
    info.header_off = F.header_off;
    info.header_len = F.header_len;
    info.trailer_off = F.trailer_off;
    info.trailer_len = F.trailer_len;
    info.num_desc = (int64_t)out.descs.size() - info.first_desc;
    (void)cur;
    chain_blocks(out, info.first_desc, info.num_desc);
    if (out.chain_tables_only && out.tables.size() > tables0) {
        // this file's mode-1 table areas, compacted to the chained blocks' (same layout
        // and 16-B alignment as snapshot's); the others' offsets are never read
        size_t w = tables0;
        for (int64_t k = info.first_desc; k < info.first_desc + info.num_desc; k++) {
            BlockDesc &d = out.descs[(size_t)k];
            if (d.kind != KIND_DSD_FAST || d.dsd_table_off < tables0) continue;
            if (d.chain_len >= 2 || (d.inherit & INH_MEMBER)) {
                const size_t bins = (size_t)d.dsd_history_bins, n = bins * 2052 + 16;
                w = (w + 15) & ~(size_t)15;
                memmove(out.tables.data() + w, out.tables.data() + d.dsd_table_off, n);
                d.dsd_table_off = w;
                w += n;
            } else {
                d.dsd_table_off = 0;
            }
        }
        out.tables.resize(w);
    }
    for (int64_t k = info.first_desc; k < info.first_desc + info.num_desc; k++) {
        BlockDesc &d = out.descs[(size_t)k];
        if (d.wvc_len && (d.kind != KIND_PCM || d.chain_len || (d.inherit & INH_MEMBER))) {
            d.crc = d.crc_lossy;  // a chain continues the lossy state: decoded as the reference does
            d.wvc_len = 0;
            d.wvc_off = 0;
            d.crc_lossy = 0;
        }
    }
}

}  // namespace wvg
