// sync_probe.cpp -- does the WavPack entropy decoder self-synchronise?
// (research probe for split-block speculative parsing; not part of the product)
//
// For every block of a file: decode the residual stream from the start (A),
// recording the decoder state at every word boundary.  Then start a second
// decoder (B) at a bit offset in the middle of the payload with guessed state,
// and report after how many words B's state (bit position, medians, holding
// flags, zeros_acc, channel) equals A's state at the same bit position --
// from there on B's words are exactly A's.
//
// g++ -O2 -std=c++17 -o /tmp/sync_probe scripts/sync_probe.cpp wavpackdecoder_amd/csrc/wv_framing.cpp
// python -c "from synth import corpora; open('/tmp/c2.wv','wb').write(corpora.c2(nblocks=64))"
// /tmp/sync_probe /tmp/c2.wv
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "../wavpackdecoder_amd/csrc/wv_decode_core.h"
#include "../wavpackdecoder_amd/csrc/wv_framing.h"

using namespace wvg;

struct St {
    int32_t med[6];
    int32_t h0, h1, ch;
    int64_t za;
    bool operator==(const St &o) const {
        for (int i = 0; i < 6; i++)
            if (med[i] != o.med[i]) return false;
        return h0 == o.h0 && h1 == o.h1 && ch == o.ch && za == o.za;
    }
};
static St snap(const Entropy &w, int ch) {
    St s;
    for (int c = 0; c < 2; c++)
        for (int k = 0; k < 3; k++) s.med[c * 3 + k] = w.med[c][k];
    s.h0 = w.h0;
    s.h1 = w.h1;
    s.ch = ch;
    s.za = w.zeros_acc;
    return s;
}
static uint64_t bitpos(const BitReader &r, uint64_t start) { return (r.pos - start) * 8 - (uint64_t)r.nb; }

static void init_w(Entropy &w, const BlockDesc &d) {
    for (int c = 0; c < 2; c++) {
        for (int k = 0; k < 3; k++) w.med[c][k] = d.median[c][k];
        w.slow[c] = d.slow_level[c];
        w.errlim[c] = 0;
        w.acc[c] = d.bitrate_acc[c];
        w.dlt[c] = d.bitrate_delta[c];
    }
    w.zeros_acc = 0;
    w.h0 = w.h1 = 0;
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    std::vector<uint8_t> file;
    int ch;
    while ((ch = fgetc(f)) != EOF) file.push_back((uint8_t)ch);
    fclose(f);
    FramingOutput fo;
    FileInfo info;
    frame_file(file.data(), file.size(), 0, 0, 0, 4096, fo, info);
    const int mode = argc > 2 ? atoi(argv[2]) : 0;  // B's guess: 0 block-start medians, 1 true medians, 2 A's medians 500 words earlier
    std::vector<int> hist;
    long never = 0, total = 0;
    for (const BlockDesc &d : fo.descs) {
        if (d.kind != KIND_PCM) continue;
        const bool mono = (d.flags & wvf::MONO_DATA) != 0;
        const uint32_t N = mono ? d.nframes : 2 * d.nframes;
        // A
        BitReader a;
        a.init(file.data(), d.bits_off, d.bits_len);
        Entropy w;
        init_w(w, d);
        std::unordered_map<uint64_t, std::pair<uint32_t, St>> at;  // bitpos -> (word, state before it)
        std::vector<uint64_t> pos(N + 1);
        std::vector<St> sts(N + 1);
        for (uint32_t k = 0; k < N; k++) {
            int c = mono ? 0 : (int)(k & 1);
            pos[k] = bitpos(a, d.bits_off);
            sts[k] = snap(w, c);
            at[pos[k]] = {k, sts[k]};
            int32_t v;
            if (get_word(w, a, d.flags, c, c == 0, v) != DEC_OK) break;
        }
        // B: several starts in the second half
        for (int trial = 0; trial < 8; trial++) {
            uint32_t s = N / 2 + (uint32_t)trial * (N / 20);
            if (s >= N) break;
            for (int delta : {0, 3, 17}) {
                BitReader b;
                b.init(file.data(), d.bits_off, d.bits_len);
                uint64_t target = pos[s] + (uint64_t)delta;
                for (uint64_t skipped = 0; skipped < target;) {
                    int n = (int)((target - skipped) > 24 ? 24 : (target - skipped));
                    b.getbits(n);
                    skipped += (uint64_t)n;
                }
                Entropy wb;
                init_w(wb, d);
                if (mode == 1) {
                    for (int i = 0; i < 6; i++) wb.med[i / 3][i % 3] = sts[s].med[i];
                } else if (mode == 2 && s >= 500) {
                    for (int i = 0; i < 6; i++) wb.med[i / 3][i % 3] = sts[s - 500].med[i];
                }
                int cb = (int)(s & 1) ^ (delta & 1);  // parity guess
                if (mono) cb = 0;
                int found = -1;
                for (int j = 0; j < 20000; j++) {
                    uint64_t p = bitpos(b, d.bits_off);
                    auto it = at.find(p);
                    if (it != at.end() && it->second.second == snap(wb, cb)) {
                        found = j;
                        break;
                    }
                    int32_t v;
                    if (get_word(wb, b, d.flags, cb, cb == 0, v) != DEC_OK) break;
                    if (!mono) cb ^= 1;
                }
                total++;
                if (found < 0) never++;
                else hist.push_back(found);
            }
        }
    }
    std::sort(hist.begin(), hist.end());
    auto q = [&](double x) { return hist.empty() ? -1 : hist[(size_t)(x * (hist.size() - 1))]; };
    printf("trials=%ld synced=%zu never(20000 words)=%ld  words-to-sync: p10=%d p50=%d p90=%d p99=%d max=%d\n", total,
           hist.size(), never, q(0.1), q(0.5), q(0.9), q(0.99), hist.empty() ? -1 : hist.back());
    return 0;
}
