// Issue-cost microbenchmarks for one wave (scalar-heavy parser design).
// hipcc --offload-arch=gfx950 -O3 issue.hip -o issue && ./issue
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP100(x) x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x x
#define BENCH(name, setup, body)                                               \
    __global__ void name(long long *out) {                                    \
        asm volatile(setup ::: "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "v20", "v21", "v22", "v23", "v24", "v25", "scc", "vcc"); \
        long long t0 = clock64();                                              \
        asm volatile(REP100(body) ::: "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "v20", "v21", "v22", "v23", "v24", "v25", "scc", "vcc"); \
        long long t1 = clock64();                                              \
        if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;                       \
    }

BENCH(k_nop, "", "s_nop 0\n")
BENCH(k_sadd_dep, "s_mov_b32 s20, 0\n", "s_add_u32 s20, s20, 1\n")
BENCH(k_sadd_ind, "s_mov_b32 s20, 0\n s_mov_b32 s21, 0\n s_mov_b32 s22, 0\n s_mov_b32 s23, 0\n",
      "s_add_u32 s20, s20, 1\n s_add_u32 s21, s21, 1\n s_add_u32 s22, s22, 1\n s_add_u32 s23, s23, 1\n")
BENCH(k_smul_dep, "s_mov_b32 s20, 3\n", "s_mul_i32 s20, s20, 3\n")
BENCH(k_shr64_dep, "s_mov_b64 s[20:21], -1\n", "s_lshr_b64 s[20:21], s[20:21], 1\n")
BENCH(k_cmp_csel, "s_mov_b32 s20, 0\n s_mov_b32 s21, 5\n", "s_cmp_lt_u32 s20, s21\n s_cselect_b32 s20, s21, s20\n")
BENCH(k_ff1_dep, "s_mov_b32 s20, 5\n", "s_ff1_i32_b32 s20, s20\n")
BENCH(k_branch_taken, "", "s_branch 0\n")
BENCH(k_cbranch_nt, "s_cmp_eq_u32 0, 1\n", "s_cbranch_scc1 0\n")
BENCH(k_cbranch_t, "s_cmp_eq_u32 0, 0\n", "s_cbranch_scc1 0\n")
BENCH(k_valu_dep, "v_mov_b32 v20, 0\n", "v_add_u32 v20, v20, 1\n")
BENCH(k_rfl, "v_mov_b32 v20, 0\n", "v_add_u32 v20, 1, v20\n v_readfirstlane_b32 s20, v20\n s_add_u32 s21, s20, 1\n")
BENCH(k_wl, "s_mov_b32 s20, 7\n s_mov_b32 m0, 3\n", "v_writelane_b32 v20, s20, m0\n s_add_u32 s20, s20, 1\n")
BENCH(k_mix, "s_mov_b32 s20, 0\n v_mov_b32 v20, 0\n", "s_add_u32 s20, s20, 1\n v_add_u32 v20, v20, 1\n")
// VALU multiplies: 64-bit mad (apply_weight), 32-bit mul_lo, 24-bit mul, dependent and independent
BENCH(k_mad64_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n s_mov_b64 s[20:21], 0x200\n",
      "v_mad_i64_i32 v[20:21], s[22:23], v20, v21, s[20:21]\n")
BENCH(k_mad64_ind, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n s_mov_b64 s[20:21], 0x200\n",
      "v_mad_i64_i32 v[22:23], s[24:25], v20, v21, s[20:21]\n v_mad_i64_i32 v[24:25], s[26:27], v20, v21, s[20:21]\n")
BENCH(k_mullo_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mul_lo_u32 v20, v20, v21\n")
BENCH(k_mul24_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mul_i32_i24 v20, v20, v21\n")
BENCH(k_mad24_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n", "v_mad_i32_i24 v20, v20, v21, v21\n")

// lane-kernel patterns: lane masks through SGPRs, 64-bit shifts, LDS round trips
BENCH(k_cmp_cnd, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_cmp_gt_u32_e64 s[20:21], v20, v21\n v_cndmask_b32_e64 v20, v21, v20, s[20:21]\n")
BENCH(k_cmp_sand_cnd, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n s_mov_b64 s[24:25], -1\n",
      "v_cmp_gt_u32_e64 s[20:21], v20, v21\n s_and_b64 s[22:23], s[20:21], s[24:25]\n v_cndmask_b32_e64 v20, v21, v20, s[22:23]\n")
BENCH(k_cmp_scbr, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n",
      "v_cmp_gt_u32_e64 s[20:21], v20, v21\n s_cmp_eq_u64 s[20:21], 0\n s_cbranch_scc0 1\n s_nop 0\n v_add_u32 v20, v20, 1\n")
BENCH(k_shr64v_dep, "v_mov_b32 v20, -1\n v_mov_b32 v21, -1\n", "v_lshrrev_b64 v[20:21], 1, v[20:21]\n")
BENCH(k_ffbl_dep, "v_mov_b32 v20, 5\n", "v_ffbl_b32 v20, v20\n")
BENCH(k_cnd_vcc_dep, "v_mov_b32 v20, 3\n v_mov_b32 v21, 5\n s_mov_b64 vcc, -1\n", "v_cndmask_b32 v20, v21, v20, vcc\n")
BENCH(k_ds_dep, "v_mov_b32 v20, 0\n", "ds_read_b32 v20, v20\n s_waitcnt lgkmcnt(0)\n")
BENCH(k_valu_ind4, "v_mov_b32 v20, 0\n v_mov_b32 v21, 0\n v_mov_b32 v22, 0\n v_mov_b32 v23, 0\n",
      "v_add_u32 v20, v20, 1\n v_add_u32 v21, v21, 1\n v_add_u32 v22, v22, 1\n v_add_u32 v23, v23, 1\n")

int main() {
    long long *d;
    hipMalloc(&d, 1024 * sizeof(long long));
    long long h[1024];
    struct { const char *n; void (*k)(long long *); } ks[] = {
        {"nop", k_nop}, {"sadd_dep", k_sadd_dep}, {"sadd_ind(x4)", k_sadd_ind}, {"smul_dep", k_smul_dep},
        {"shr64_dep", k_shr64_dep}, {"cmp+cselect", k_cmp_csel}, {"ff1_dep", k_ff1_dep},
        {"s_branch", k_branch_taken}, {"cbranch_not_taken", k_cbranch_nt}, {"cbranch_taken", k_cbranch_t},
        {"valu_dep", k_valu_dep}, {"valu+rfl+salu", k_rfl}, {"writelane+sadd", k_wl}, {"salu+valu", k_mix},
        {"v_mad_i64_dep", k_mad64_dep}, {"v_mad_i64_ind(x2)", k_mad64_ind}, {"v_mul_lo_u32_dep", k_mullo_dep},
        {"v_mul_i32_i24_dep", k_mul24_dep}, {"v_mad_i32_i24_dep", k_mad24_dep},
        {"v_cmp->v_cndmask", k_cmp_cnd}, {"v_cmp->s_and->v_cnd", k_cmp_sand_cnd}, {"v_cmp->s_cbranch(x5)", k_cmp_scbr},
        {"v_lshrrev_b64_dep", k_shr64v_dep}, {"v_ffbl_dep", k_ffbl_dep}, {"v_cndmask_vcc_dep", k_cnd_vcc_dep},
        {"ds_read_dep", k_ds_dep}, {"valu_ind(x4)", k_valu_ind4}};
    for (auto &k : ks) {
        for (int nb : {1, 1024, 2048}) {
            for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k.k, dim3(nb), dim3(64), 0, 0, d);
            hipDeviceSynchronize();
            hipMemcpy(h, d, sizeof(long long) * (nb < 1024 ? nb : 1024), hipMemcpyDeviceToHost);
            printf("%-20s blocks=%4d  cycles/rep=%.2f\n", k.n, nb, h[0] / 100.0);
        }
    }
    return 0;
}
