// Issue-cost microbenchmarks for one wave (scalar-heavy parser design, lane-kernel
// VALU patterns) and for two waves sharing a SIMD.
// hipcc --offload-arch=gfx950 -O3 issue.hip -o issue && ./issue
// Prints cycles per repetition of each body (100 repetitions timed with s_memtime
// via clock64), for 1 workgroup of 64 threads (one wave alone on the chip) and for
// 256 / 512-thread workgroups (one / two waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP100(x) x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x
#define CLOB "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "scc", "vcc"
#define BENCH(name, setup, body)                                               \
    __global__ void name(long long *out) {                                    \
        asm volatile(setup ::: CLOB);                                          \
        long long t0 = clock64();                                              \
        asm volatile(REP100(body) ::: CLOB);                                   \
        long long t1 = clock64();                                              \
        if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0; \
    }

BENCH(k_nop, "", "s_nop 0\n")
BENCH(k_sadd_dep, "s_mov_b32 s20, 0\n", "s_add_u32 s20, s20, 1\n")
BENCH(k_sadd_ind, "s_mov_b32 s20, 0\n s_mov_b32 s21, 0\n s_mov_b32 s22, 0\n s_mov_b32 s23, 0\n",
      "s_add_u32 s20, s20, 1\n s_add_u32 s21, s21, 1\n s_add_u32 s22, s22, 1\n s_add_u32 s23, s23, 1\n")
BENCH(k_branch_taken, "", "s_branch 0\n")
BENCH(k_cbranch_nt, "s_cmp_eq_u32 0, 1\n", "s_cbranch_scc1 0\n")
BENCH(k_valu_dep, "v_mov_b32 v20, 0\n", "v_add_u32 v20, v20, 1\n")
BENCH(k_valu_ind4, "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n",
      "v_add_u32 v20, v20, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v22, v22, 1\n v_add_u32 v23, v23, 1\n")
BENCH(k_salu_valu, "s_mov_b32 s20, 0\n v_mov_b32 v20, 0\n", "s_add_u32 s20, s20, 1\n v_add_u32 v20, v20, 1\n")
// the lane parser's instruction mix
BENCH(k_shr64_dep, "v_mov_b32 v20, -1\n v_mov_b32 v21, -1\n v_mov_b32 v22, 1\n", "v_lshrrev_b64 v[20:21], v22, v[20:21]\n")
BENCH(k_shr64_ind, "v_mov_b32 v20, -1\n v_mov_b32 v21, -1\n v_mov_b32 v22, 1\n",
      "v_lshrrev_b64 v[24:25], v22, v[20:21]\n v_lshrrev_b64 v[26:27], v22, v[20:21]\n")
BENCH(k_shl64_dep, "v_mov_b32 v20, 1\n v_mov_b32 v21, 0\n v_mov_b32 v22, 1\n", "v_lshlrev_b64 v[20:21], v22, v[20:21]\n")
BENCH(k_lshladd64_dep, "v_mov_b32 v20, 1\n v_mov_b32 v21, 0\n v_mov_b32 v22, 1\n", "v_lshl_add_u64 v[20:21], v[20:21], 1, v[20:21]\n")
BENCH(k_alignbit_dep, "v_mov_b32 v20, 5\n v_mov_b32 v21, 7\n v_mov_b32 v22, 3\n", "v_alignbit_b32 v20, v21, v20, v22\n")
BENCH(k_bitop3_dep, "v_mov_b32 v20, 5\n v_mov_b32 v21, 7\n", "v_bitop3_b32 v20, v20, v21, v20 bitop3:0xc8\n")
BENCH(k_add3_dep, "v_mov_b32 v20, 5\n v_mov_b32 v21, 7\n", "v_add3_u32 v20, v20, v21, v20\n")
BENCH(k_bfe_dep, "v_mov_b32 v20, 5\n", "v_bfe_u32 v20, v20, 1, 7\n")
BENCH(k_ffbl_dep, "v_mov_b32 v20, 5\n", "v_ffbl_b32 v20, v20\n")
BENCH(k_ffbh_dep, "v_mov_b32 v20, 5\n", "v_ffbh_u32 v20, v20\n")
BENCH(k_min_dep, "v_mov_b32 v20, 5\n v_mov_b32 v21, 7\n", "v_min_u32 v20, v20, v21\n")
BENCH(k_med3_dep, "v_mov_b32 v20, 5\n v_mov_b32 v21, 7\n", "v_med3_i32 v20, v20, v21, 3\n")
BENCH(k_mul24_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mul_u32_u24 v20, v20, v21\n")
BENCH(k_mad24_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mad_i32_i24 v20, v20, v21, v21\n")
BENCH(k_mullo_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mul_lo_u32 v20, v20, v21\n")
BENCH(k_mullo_ind, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mul_lo_u32 v22, v20, v21\n v_mul_lo_u32 v23, v20, v21\n")
BENCH(k_cmp_cnd_vcc, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_cmp_gt_u32 vcc, v20, v21\n v_cndmask_b32 v20, v21, v20, vcc\n")
BENCH(k_cmp_cnd_sgpr, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_cmp_gt_u32_e64 s[20:21], v20, v21\n v_cndmask_b32_e64 v20, v21, v20, s[20:21]\n")
BENCH(k_cmp_addc, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_cmp_gt_u32 vcc, v20, v21\n v_addc_co_u32 v20, vcc, 0, v20, vcc\n")
BENCH(k_cmp_sand_cnd, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n s_mov_b64 s[24:25], -1\n",
      "v_cmp_gt_u32_e64 s[20:21], v20, v21\n s_and_b64 s[22:23], s[20:21], s[24:25]\n v_cndmask_b32_e64 v20, v21, v20, s[22:23]\n")
BENCH(k_ashr_mask, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_sub_u32 v22, v20, v21\n v_ashrrev_i32 v22, 31, v22\n v_and_b32 v20, v22, v21\n")
BENCH(k_ds_dep, "v_mov_b32 v20, 0\n", "ds_read_b32 v20, v20\n s_waitcnt lgkmcnt(0)\n")
BENCH(k_ds_hidden, "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n",
      "ds_read_b32 v22, v20\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v21, v21, 1\n s_waitcnt lgkmcnt(0)\n v_add_u32 v21, v21, v22\n")
BENCH(k_dswrite, "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n", "ds_write_b32 v20, v21\n")
BENCH(k_dswrite64, "v_mov_b32 v20, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n", "ds_write_b64 v20, v[22:23]\n")
BENCH(k_pk_add_f32, "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n",
      "v_pk_add_f32 v[20:21], v[20:21], v[22:23]\n")

// the decorr passes' apply_weight: a 64-bit product then the 10-bit shift
BENCH(k_madi64_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 0\n v_mov_b32 v22, 5\n",
      "v_mad_i64_i32 v[20:21], s[20:21], v20, v22, 0\n")
BENCH(k_madi64_ind, "v_mov_b32 v20, 3\n v_mov_b32 v21, 0\n v_mov_b32 v22, 5\n",
      "v_mad_i64_i32 v[24:25], s[20:21], v20, v22, 0\n v_mad_i64_i32 v[26:27], s[22:23], v20, v22, 0\n")
BENCH(k_aw64_chain, "v_mov_b32 v20, 3\n v_mov_b32 v21, 0\n v_mov_b32 v22, 5\n",
      "v_mad_i64_i32 v[24:25], s[20:21], v20, v22, 0\n v_alignbit_b32 v20, v25, v24, 10\n")
BENCH(k_aw24_chain, "v_mov_b32 v20, 3\n v_mov_b32 v21, 0\n v_mov_b32 v22, 5\n s_movk_i32 s24, 0x200\n",
      "v_ashrrev_i32 v24, 12, v20\n v_and_b32 v25, 0xfff, v20\n v_mul_i32_i24 v24, v22, v24\n v_mad_i32_i24 v25, v22, v25, s24\n v_ashrrev_i32 v25, 10, v25\n v_lshl_add_u32 v20, v24, 2, v25\n")
BENCH(k_cbranch_taken, "s_cmp_eq_u32 0, 0\n", "s_cbranch_scc1 0\n")

typedef void (*kfn)(long long *);
int main() {
    long long *d;
    (void)hipMalloc(&d, 1024 * 8 * sizeof(long long));
    static long long h[1024 * 8];
    struct { const char *n; kfn k; } ks[] = {
        {"s_nop", k_nop}, {"s_add dep", k_sadd_dep}, {"s_add ind x4", k_sadd_ind}, {"s_branch", k_branch_taken},
        {"s_cbranch not taken", k_cbranch_nt}, {"v_add dep", k_valu_dep}, {"v_add ind x4", k_valu_ind4},
        {"s_add+v_add", k_salu_valu}, {"v_lshrrev_b64 dep", k_shr64_dep}, {"v_lshrrev_b64 ind x2", k_shr64_ind},
        {"v_lshlrev_b64 dep", k_shl64_dep}, {"v_lshl_add_u64 dep", k_lshladd64_dep}, {"v_alignbit dep", k_alignbit_dep},
        {"v_bitop3 dep", k_bitop3_dep}, {"v_add3 dep", k_add3_dep}, {"v_bfe_u32 dep", k_bfe_dep},
        {"v_ffbl dep", k_ffbl_dep}, {"v_ffbh dep", k_ffbh_dep}, {"v_min_u32 dep", k_min_dep}, {"v_med3 dep", k_med3_dep},
        {"v_mul_u32_u24 dep", k_mul24_dep}, {"v_mad_i32_i24 dep", k_mad24_dep}, {"v_mul_lo_u32 dep", k_mullo_dep},
        {"v_mul_lo_u32 ind x2", k_mullo_ind}, {"v_mad_i64_i32 dep", k_madi64_dep}, {"v_mad_i64_i32 ind x2", k_madi64_ind},
        {"aw: mad_i64+alignbit chain", k_aw64_chain}, {"aw: 24-bit split chain (6)", k_aw24_chain},
        {"s_cbranch taken", k_cbranch_taken}, {"v_cmp->v_cndmask vcc", k_cmp_cnd_vcc},
        {"v_cmp->v_cndmask sgpr", k_cmp_cnd_sgpr}, {"v_cmp->v_addc vcc", k_cmp_addc},
        {"v_cmp->s_and->v_cndmask", k_cmp_sand_cnd}, {"v_sub,v_ashr,v_and", k_ashr_mask},
        {"ds_read dep", k_ds_dep}, {"ds_read + 16 v_add", k_ds_hidden}, {"ds_write_b32", k_dswrite},
        {"ds_write_b64", k_dswrite64}, {"v_pk_add_f32 dep", k_pk_add_f32}};
    for (auto &k : ks) {
        printf("%-26s", k.n);
        // 1 wave alone; 1024 workgroups x 1 wave; 256-thread (1 wave per SIMD) and
        // 512-thread (2 waves per SIMD) workgroups, 256 of them
        struct { int nb, nt; } cfg[] = {{1, 64}, {1024, 64}, {256, 256}, {256, 512}};
        for (auto c : cfg) {
            for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k.k, dim3(c.nb), dim3(c.nt), 1024, 0, d);  // (1 KiB of LDS for the ds_ bodies, address 0)
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h, d, sizeof(long long) * 8 * c.nb, hipMemcpyDeviceToHost);
            double s = 0;
            int n = 0;
            for (int b = 0; b < c.nb; b++)
                for (int w = 0; w < c.nt / 64; w++) s += h[b * 8 + w], n++;
            printf("  %4dx%3d %7.2f", c.nb, c.nt, s / n / 100.0);
        }
        printf("\n");
    }
    return 0;
}
