// VALU throughput probe: wave-instructions per SIMD-cycle-equivalent for the
// integer forms the decode loops use.  Each thread runs 8 independent chains
// of one instruction (inline asm, 256 unrolled), many waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define OP_KERNEL(name, body)                                                         \
  __global__ void __launch_bounds__(256) name(uint32_t *out, int iters) {             \
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,     \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, s = a0 | 1;                          \
    uint64_t q0 = a0, q1 = a1, q2 = a2, q3 = a3;                                        \
    for (int i = 0; i < iters; i++) { REP8(REP8(body)) }                                \
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(q0 ^ q1 ^ q2 ^ q3)) == 0x12345) \
      out[blockIdx.x] = 1;                                                              \
  }

OP_KERNEL(k_add, asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_mul24, asm volatile("v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_bfe, asm volatile("v_bfe_u32 %0, %0, %8, 5\n v_bfe_u32 %1, %1, %8, 5\n v_bfe_u32 %2, %2, %8, 5\n v_bfe_u32 %3, %3, %8, 5\n v_bfe_u32 %4, %4, %8, 5\n v_bfe_u32 %5, %5, %8, 5\n v_bfe_u32 %6, %6, %8, 5\n v_bfe_u32 %7, %7, %8, 5" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_shl64, asm volatile("v_lshlrev_b64 %0, %4, %0\n v_lshlrev_b64 %1, %4, %1\n v_lshlrev_b64 %2, %4, %2\n v_lshlrev_b64 %3, %4, %3" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(s));)
OP_KERNEL(k_mad64, asm volatile("v_mad_u64_u32 %0, vcc, %4, %4, %0\n v_mad_u64_u32 %1, vcc, %4, %4, %1\n v_mad_u64_u32 %2, vcc, %4, %4, %2\n v_mad_u64_u32 %3, vcc, %4, %4, %3" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(s) : "vcc");)
OP_KERNEL(k_cndmask, asm volatile("v_cmp_gt_u32 vcc, %8, %0\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %1, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s) : "vcc");)

OP_KERNEL(k_cnd_only, asm volatile("v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %0, vcc\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s) : "vcc");)
OP_KERNEL(k_cmp_only, asm volatile("v_cmp_gt_u32 vcc, %8, %0\n v_cmp_gt_u32 vcc, %8, %1\n v_cmp_gt_u32 vcc, %8, %2\n v_cmp_gt_u32 vcc, %8, %3\n v_cmp_gt_u32 vcc, %8, %4\n v_cmp_gt_u32 vcc, %8, %5\n v_cmp_gt_u32 vcc, %8, %6\n v_cmp_gt_u32 vcc, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s) : "vcc");)
OP_KERNEL(k_cnd_sgpr, asm volatile("v_cmp_gt_u32 s[40:41], %8, %0\n v_cndmask_b32_e64 %1, %1, %2, s[40:41]\n v_cndmask_b32_e64 %2, %2, %3, s[40:41]\n v_cndmask_b32_e64 %3, %3, %4, s[40:41]\n v_cndmask_b32_e64 %4, %4, %5, s[40:41]\n v_cndmask_b32_e64 %5, %5, %6, s[40:41]\n v_cndmask_b32_e64 %6, %6, %7, s[40:41]\n v_cndmask_b32_e64 %7, %7, %1, s[40:41]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s) : "s40", "s41");)
OP_KERNEL(k_max, asm volatile("v_max_u32 %0, %0, %8\n v_max_u32 %1, %1, %8\n v_max_u32 %2, %2, %8\n v_max_u32 %3, %3, %8\n v_max_u32 %4, %4, %8\n v_max_u32 %5, %5, %8\n v_max_u32 %6, %6, %8\n v_max_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_add3, asm volatile("v_add3_u32 %0, %0, %8, %1\n v_add3_u32 %1, %1, %8, %2\n v_add3_u32 %2, %2, %8, %3\n v_add3_u32 %3, %3, %8, %4\n v_add3_u32 %4, %4, %8, %5\n v_add3_u32 %5, %5, %8, %6\n v_add3_u32 %6, %6, %8, %7\n v_add3_u32 %7, %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_lshr, asm volatile("v_lshrrev_b32 %0, %8, %0\n v_lshrrev_b32 %1, %8, %1\n v_lshrrev_b32 %2, %8, %2\n v_lshrrev_b32 %3, %8, %3\n v_lshrrev_b32 %4, %8, %4\n v_lshrrev_b32 %5, %8, %5\n v_lshrrev_b32 %6, %8, %6\n v_lshrrev_b32 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_lshr_e64, asm volatile("v_lshrrev_b32_e64 %0, %8, %0\n v_lshrrev_b32_e64 %1, %8, %1\n v_lshrrev_b32_e64 %2, %8, %2\n v_lshrrev_b32_e64 %3, %8, %3\n v_lshrrev_b32_e64 %4, %8, %4\n v_lshrrev_b32_e64 %5, %8, %5\n v_lshrrev_b32_e64 %6, %8, %6\n v_lshrrev_b32_e64 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)

OP_KERNEL(k_mulhi24, asm volatile("v_mul_hi_u32_u24 %0, %0, %8\n v_mul_hi_u32_u24 %1, %1, %8\n v_mul_hi_u32_u24 %2, %2, %8\n v_mul_hi_u32_u24 %3, %3, %8\n v_mul_hi_u32_u24 %4, %4, %8\n v_mul_hi_u32_u24 %5, %5, %8\n v_mul_hi_u32_u24 %6, %6, %8\n v_mul_hi_u32_u24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_mul_i24, asm volatile("v_mul_i32_i24 %0, %0, %8\n v_mul_i32_i24 %1, %1, %8\n v_mul_i32_i24 %2, %2, %8\n v_mul_i32_i24 %3, %3, %8\n v_mul_i32_i24 %4, %4, %8\n v_mul_i32_i24 %5, %5, %8\n v_mul_i32_i24 %6, %6, %8\n v_mul_i32_i24 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_lshl_or, asm volatile("v_lshl_or_b32 %0, %0, 8, %8\n v_lshl_or_b32 %1, %1, 8, %8\n v_lshl_or_b32 %2, %2, 8, %8\n v_lshl_or_b32 %3, %3, 8, %8\n v_lshl_or_b32 %4, %4, 8, %8\n v_lshl_or_b32 %5, %5, 8, %8\n v_lshl_or_b32 %6, %6, 8, %8\n v_lshl_or_b32 %7, %7, 8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_add_lshl, asm volatile("v_add_lshl_u32 %0, %0, %8, 4\n v_add_lshl_u32 %1, %1, %8, 4\n v_add_lshl_u32 %2, %2, %8, 4\n v_add_lshl_u32 %3, %3, %8, 4\n v_add_lshl_u32 %4, %4, %8, 4\n v_add_lshl_u32 %5, %5, %8, 4\n v_add_lshl_u32 %6, %6, %8, 4\n v_add_lshl_u32 %7, %7, %8, 4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_and, asm volatile("v_and_b32 %0, %8, %0\n v_and_b32 %1, %8, %1\n v_and_b32 %2, %8, %2\n v_and_b32 %3, %8, %3\n v_and_b32 %4, %8, %4\n v_and_b32 %5, %8, %5\n v_and_b32 %6, %8, %6\n v_and_b32 %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_perm, asm volatile("v_perm_b32 %0, %0, %8, %8\n v_perm_b32 %1, %1, %8, %8\n v_perm_b32 %2, %2, %8, %8\n v_perm_b32 %3, %3, %8, %8\n v_perm_b32 %4, %4, %8, %8\n v_perm_b32 %5, %5, %8, %8\n v_perm_b32 %6, %6, %8, %8\n v_perm_b32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_dot2u16, asm volatile("v_dot2_u32_u16 %0, %0, %8, %0\n v_dot2_u32_u16 %1, %1, %8, %1\n v_dot2_u32_u16 %2, %2, %8, %2\n v_dot2_u32_u16 %3, %3, %8, %3\n v_dot2_u32_u16 %4, %4, %8, %4\n v_dot2_u32_u16 %5, %5, %8, %5\n v_dot2_u32_u16 %6, %6, %8, %6\n v_dot2_u32_u16 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_pk_mul_lo, asm volatile("v_pk_mul_lo_u16 %0, %0, %8\n v_pk_mul_lo_u16 %1, %1, %8\n v_pk_mul_lo_u16 %2, %2, %8\n v_pk_mul_lo_u16 %3, %3, %8\n v_pk_mul_lo_u16 %4, %4, %8\n v_pk_mul_lo_u16 %5, %5, %8\n v_pk_mul_lo_u16 %6, %6, %8\n v_pk_mul_lo_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_pk_add_u16, asm volatile("v_pk_add_u16 %0, %0, %8\n v_pk_add_u16 %1, %1, %8\n v_pk_add_u16 %2, %2, %8\n v_pk_add_u16 %3, %3, %8\n v_pk_add_u16 %4, %4, %8\n v_pk_add_u16 %5, %5, %8\n v_pk_add_u16 %6, %6, %8\n v_pk_add_u16 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_cvt_ubyte, asm volatile("v_cvt_f32_ubyte1 %0, %0\n v_cvt_f32_ubyte1 %1, %1\n v_cvt_f32_ubyte1 %2, %2\n v_cvt_f32_ubyte1 %3, %3\n v_cvt_f32_ubyte1 %4, %4\n v_cvt_f32_ubyte1 %5, %5\n v_cvt_f32_ubyte1 %6, %6\n v_cvt_f32_ubyte1 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_fmul, asm volatile("v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_mad_u24, asm volatile("v_mad_u32_u24 %0, %0, %8, %0\n v_mad_u32_u24 %1, %1, %8, %1\n v_mad_u32_u24 %2, %2, %8, %2\n v_mad_u32_u24 %3, %3, %8, %3\n v_mad_u32_u24 %4, %4, %8, %4\n v_mad_u32_u24 %5, %5, %8, %5\n v_mad_u32_u24 %6, %6, %8, %6\n v_mad_u32_u24 %7, %7, %8, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_alignbyte, asm volatile("v_alignbyte_b32 %0, %0, %8, %8\n v_alignbyte_b32 %1, %1, %8, %8\n v_alignbyte_b32 %2, %2, %8, %8\n v_alignbyte_b32 %3, %3, %8, %8\n v_alignbyte_b32 %4, %4, %8, %8\n v_alignbyte_b32 %5, %5, %8, %8\n v_alignbyte_b32 %6, %6, %8, %8\n v_alignbyte_b32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_bfe3, asm volatile("v_bfe_u32 %0, %0, 8, 8\n v_bfe_u32 %1, %1, 8, 8\n v_bfe_u32 %2, %2, 8, 8\n v_bfe_u32 %3, %3, 8, 8\n v_bfe_u32 %4, %4, 8, 8\n v_bfe_u32 %5, %5, 8, 8\n v_bfe_u32 %6, %6, 8, 8\n v_bfe_u32 %7, %7, 8, 8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)
OP_KERNEL(k_cvt_pk_u8, asm volatile("v_cvt_pk_u8_f32 %0, %0, 1, %0\n v_cvt_pk_u8_f32 %1, %1, 1, %1\n v_cvt_pk_u8_f32 %2, %2, 1, %2\n v_cvt_pk_u8_f32 %3, %3, 1, %3\n v_cvt_pk_u8_f32 %4, %4, 1, %4\n v_cvt_pk_u8_f32 %5, %5, 1, %5\n v_cvt_pk_u8_f32 %6, %6, 1, %6\n v_cvt_pk_u8_f32 %7, %7, 1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(s));)

int main() {
  uint32_t *out;
  hipMalloc(&out, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int dev;
  hipGetDevice(&dev);
  int clk;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  struct { const char *n; void (*k)(uint32_t *, int); int per_iter; } ks[] = {
      {"v_add_u32", k_add, 512}, {"v_mul_u32_u24", k_mul24, 512}, {"v_mul_lo_u32", k_mullo, 512},
      {"v_bfe_u32", k_bfe, 512}, {"v_lshlrev_b64", k_shl64, 256}, {"v_mad_u64_u32", k_mad64, 256},
      {"v_cmp+v_cndmask (8 per 8)", k_cndmask, 512}, {"v_cndmask vcc only", k_cnd_only, 512},
      {"v_cmp -> vcc only", k_cmp_only, 512}, {"v_cmp+v_cndmask_e64 sgpr", k_cnd_sgpr, 512},
      {"v_max_u32", k_max, 512}, {"v_add3_u32", k_add3, 512}, {"v_lshrrev_b32 (e32)", k_lshr, 512},
      {"v_lshrrev_b32_e64", k_lshr_e64, 512}, {"v_mul_hi_u32_u24", k_mulhi24, 512}, {"v_mul_i32_i24", k_mul_i24, 512}, {"v_lshl_or_b32", k_lshl_or, 512}, {"v_add_lshl_u32", k_add_lshl, 512}, {"v_and_b32", k_and, 512}, {"v_perm_b32", k_perm, 512}, {"v_dot2_u32_u16", k_dot2u16, 512}, {"v_pk_mul_lo_u16", k_pk_mul_lo, 512}, {"v_pk_add_u16", k_pk_add_u16, 512}, {"v_cvt_f32_ubyte1", k_cvt_ubyte, 512}, {"v_mul_f32", k_fmul, 512}, {"v_mad_u32_u24", k_mad_u24, 512}, {"v_alignbyte_b32", k_alignbyte, 512}, {"v_bfe_u32", k_bfe3, 512}, {"v_cvt_pk_u8_f32", k_cvt_pk_u8, 512}};
  const int blocks = 256 * 8 * 4, iters = 64;  // 8 waves per SIMD
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double winstr = (double)blocks * 4 * iters * k.per_iter;  // wave-instructions
    double per_simd_s = winstr / 1024.0 / (ms * 1e-3);
    printf("%-28s %8.3f ms  %.3f wave-instr/ns per SIMD  (%.2f cycles each at %.2f GHz nominal)\n", k.n, ms,
           per_simd_s * 1e-9, clk * 1e3 / per_simd_s, clk / 1e6);
  }
  return 0;
}
