// Cycle cost of the parser's hot word sequence vs simple instruction streams,
// one wave (not part of the product).
// hipcc --offload-arch=gfx950 -O3 word.hip -o word && ./word
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP10(x) x x x x x x x x x x
#define REP100(x) REP10(REP10(x))
#define CLOB "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", \
             "s34", "s35", "s36", "s37", "s38", "s39", "v20", "scc", "vcc", "m0"
#define BENCH(name, setup, body, tail)                                          \
    __global__ void name(long long *out) {                                     \
        asm volatile(setup ::: CLOB);                                           \
        long long t0 = clock64();                                               \
        asm volatile(body tail ::: CLOB);                                       \
        long long t1 = clock64();                                               \
        if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;                        \
    }

// registers: vcc window, s20 nb, s21 h0, s22 h1, s23 m0, s24 t0, s25 u, s26 ones, s27 c1, s28 mc,
// s29 z, s30 t, s31 ex, s32 v, s33 n1
#define SETUP "s_mov_b64 vcc, 0x0\n s_mov_b32 s20, 40\n s_mov_b32 s21, 0\n s_mov_b32 s22, 0\n s_movk_i32 s23, 0x400\n s_mov_b32 m0, 0\n"
// case-0 word with the window refreshed to all-zero bits each time (u = 0, short code)
#define WORD                                                                   \
    "s_mov_b32 s20, 40\n s_mov_b64 vcc, 0\n s_movk_i32 s23, 0x400\n"            \
    "s_cmp_lt_u32 s20, 32\n s_cbranch_scc1 LEND_%=\n"                          \
    "s_orn2_b32 s24, 0x10000, vcc_lo\n s_ff1_i32_b32 s25, s24\n"               \
    "s_cmp_lg_u32 s21, 0\n s_cselect_b32 s25, 0, s25\n"                        \
    "s_lshr_b32 s26, s25, 1\n s_add_u32 s26, s26, s22\n s_and_b32 s22, s25, 1\n" \
    "s_add_u32 s27, s25, 1\n s_sub_u32 s27, s27, s21\n s_xor_b32 s24, s22, 1\n s_sub_u32 s21, s24, s21\n" \
    "s_mov_b32 s21, 0\n s_mov_b32 s22, 0\n"                                    \
    "s_cmp_lg_u32 s26, 0\n s_cbranch_scc1 LEND_%=\n"                           \
    "s_lshr_b32 s28, s23, 4\n s_add_i32 s24, s23, 0x7e\n s_ashr_i32 s24, s24, 6\n s_and_b32 s24, s24, -2\n s_sub_i32 s23, s23, s24\n" \
    "s_or_b32 s24, s28, 1\n s_flbit_i32_b32 s29, s24\n s_lshr_b32 s30, vcc_lo, s27\n s_lshr_b32 s31, -1, s29\n" \
    "s_sub_u32 s31, s31, s28\n s_lshr_b32 s24, 0x7fffffff, s29\n s_and_b32 s32, s30, s24\n s_sub_u32 s33, 31, s29\n" \
    "s_cmp_lt_u32 s32, s31\n s_cbranch_scc1 1f\n"                           \
    "s_branch LEND_%=\n"                                                      \
    "1:\n"
#define WORDTAIL                                                               \
    "s_bitcmp1_b32 s30, s33\n s_cselect_b32 s24, -1, 0\n s_xor_b32 s32, s32, s24\n" \
    "s_add_u32 s33, s33, s27\n s_add_u32 s33, s33, 1\n s_lshr_b64 vcc, vcc, s33\n s_sub_u32 s20, s20, s33\n" \
    "v_writelane_b32 v20, s32, m0\n s_add_u32 m0, m0, 1\n s_and_b32 m0, m0, 63\n"

// one word = WORD + WORDTAIL (the taken branch to LS is part of it: see word_nobr)
__global__ void k_word(long long *out) {
    asm volatile(SETUP ::: CLOB);
    long long t0 = clock64();
    asm volatile(REP10(WORD WORDTAIL) "LEND_%=:\n" ::: CLOB);
    long long t1 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}
BENCH(k_sadd_dep, "s_mov_b32 s20, 0\n", REP100("s_add_u32 s20, s20, 1\n"), "")
BENCH(k_sadd_lit, "s_mov_b32 s20, 0\n", REP100("s_add_u32 s20, s20, 0x12345\n"), "")
BENCH(k_lshr64, "s_mov_b64 vcc, -1\n s_mov_b32 s20, 1\n", REP100("s_lshr_b64 vcc, vcc, s20\n"), "")
BENCH(k_bitcmp_csel, "s_mov_b32 s20, 5\n s_mov_b32 s21, 2\n",
      REP100("s_bitcmp1_b32 s20, s21\n s_cselect_b32 s22, -1, 0\n"), "")
BENCH(k_wl, "s_mov_b32 s20, 7\n s_mov_b32 m0, 3\n", REP100("v_writelane_b32 v20, s20, m0\n s_add_u32 m0, m0, 1\n s_and_b32 m0, m0, 63\n"), "")
BENCH(k_flbit, "s_mov_b32 s20, 7\n", REP100("s_flbit_i32_b32 s21, s20\n s_lshr_b32 s22, -1, s21\n"), "")
BENCH(k_vccops, "s_mov_b64 vcc, -1\n s_mov_b32 s20, 1\n",
      REP100("s_lshr_b32 s21, vcc_lo, s20\n s_orn2_b32 s22, 0x10000, vcc_lo\n"), "")

int main() {
    long long *d;
    hipMalloc(&d, 4096 * sizeof(long long));
    long long h[4096];
    struct { const char *n; void (*k)(long long *); double per; } ks[] = {
        {"word(case0,10x)", k_word, 10}, {"sadd_dep", k_sadd_dep, 100}, {"sadd_literal", k_sadd_lit, 100},
        {"lshr_b64 vcc", k_lshr64, 100}, {"bitcmp+cselect", k_bitcmp_csel, 100},
        {"writelane+add+and m0", k_wl, 100}, {"flbit+lshr", k_flbit, 100}, {"vcc_lo srcs", k_vccops, 100}};
    for (auto &k : ks) {
        for (int nb : {1, 1024, 2048}) {
            for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k.k, dim3(nb), dim3(64), 0, 0, d);
            hipDeviceSynchronize();
            hipMemcpy(h, d, sizeof(long long) * nb, hipMemcpyDeviceToHost);
            double mx = 0, sum = 0;
            for (int i = 0; i < nb; i++) { sum += h[i]; mx = h[i] > mx ? h[i] : mx; }
            printf("%-22s blocks=%4d  cycles/unit: mean=%.1f max=%.1f\n", k.n, nb, sum / nb / k.per, mx / k.per);
        }
    }
    return 0;
}
