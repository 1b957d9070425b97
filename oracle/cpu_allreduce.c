/*
 * ORACLE (test infrastructure only) — host OpenMP AllReduce, the CPU baseline of bench.py.
 *
 * The reference has no CPU implementation of the collective; this is a
 * C port of what its all-pairs LL schedule computes, used only as the timed cpu_baseline leg
 * and as a C cross-check of oracle/sim.py.  For n rank buffers x_0..x_{n-1} of `count`
 * elements the all-pairs LL result for the chunk owned by rank r is
 *     ((x_r (+) x_{p0}) (+) x_{p1}) ...   with p ascending, p != r
 * (dst-first LL reduce, prims_ll.h:347-362, scratch slots in ascending peer order); the
 * owner of element i is r = (i / (count / ncpl) / n) % n for the n x n chunk grid of one
 * instance (msccl_amd/xmlgen.py allreduce_allpairs).  fp16/bf16 are accumulated per step in
 * fp32 and rounded (RNE) after every addition, fp16 clamped to +-65504 (reduce_kernel.h:244-303).
 * Work is split over OpenMP threads in 64-byte blocks; every rank buffer receives the result.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

static inline float bf16_to_f32(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static inline float f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
  if (e == 0) {
    if (m == 0) u = sign;
    else { /* subnormal: normalise */
      e = 127 - 15 + 1;
      while (!(m & 0x400)) { m <<= 1; e--; }
      u = sign | (e << 23) | ((m & 0x3ff) << 13);
    }
  } else if (e == 31) u = sign | 0x7f800000u | (m << 13);
  else u = sign | ((e + 127 - 15) << 23) | (m << 13);
  float f;
  memcpy(&f, &u, 4);
  return f;
}
/* round-to-nearest-even f32 -> f16 (overflow -> inf) */
static inline uint16_t f32_to_f16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  uint32_t sign = (u >> 16) & 0x8000, a = u & 0x7fffffffu;
  if (a > 0x7f800000u) return (uint16_t)(sign | 0x7e00);
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00);  /* >= 65520 rounds to inf */
  if (a < 0x38800000u) {                                    /* f16 subnormal or zero */
    if (a < 0x33000000u) return (uint16_t)sign;             /* < 2^-25: rounds to 0 (ties to even) */
    uint32_t e = a >> 23, m = (a & 0x7fffff) | 0x800000;
    uint32_t sh = 126 - e;                                  /* f16 ulp 2^-24: m16 = M >> (126-e) */
    uint32_t res = m >> sh, rem = m & ((1u << sh) - 1), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (res & 1))) res++;
    return (uint16_t)(sign | res);
  }
  uint32_t res = (a - 0x38000000u) >> 13, rem = a & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (res & 1))) res++;
  return (uint16_t)(sign | res);
}
static inline uint16_t f16_add_clamp(uint16_t a, uint16_t b) {
  uint16_t r = f32_to_f16(f16_to_f32(a) + f16_to_f32(b));
  if ((r & 0x7fff) > 0x7c00) return 0xfbff;   /* NaN -> -65504 (hmax then hmin) */
  if (r == 0x7c00) return 0x7bff;             /* +inf -> 65504 */
  if (r == 0xfc00) return 0xfbff;             /* -inf -> -65504 */
  return r;
}

/* dtype: 7 = fp32, 6 = fp16, 9 = bf16.  bufs[r] points at rank r's count elements (in place).
 * chunk = elements per MSCCL chunk (count / nchunksperloop); returns threads used. */
int cpu_allreduce_allpairs(void** bufs, int n, long count, long chunk, int dtype) {
  int used = 1;
  const long block = 64;  /* bytes per work item */
  long esz = dtype == 7 ? 4 : 2;
  long per = block / esz;
  long nblk = (count + per - 1) / per;
#pragma omp parallel
  {
#pragma omp single
    used = omp_get_num_threads();
#pragma omp for schedule(static)
    for (long b = 0; b < nblk; b++) {
      long i0 = b * per, i1 = i0 + per < count ? i0 + per : count;
      for (long i = i0; i < i1; i++) {
        int r = (int)((i / chunk / n) % n);
        if (dtype == 7) {
          float acc = ((float*)bufs[r])[i];
          for (int p = 0; p < n; p++)
            if (p != r) acc = acc + ((float*)bufs[p])[i];
          for (int p = 0; p < n; p++) ((float*)bufs[p])[i] = acc;
        } else if (dtype == 6) {
          uint16_t acc = ((uint16_t*)bufs[r])[i];
          for (int p = 0; p < n; p++)
            if (p != r) acc = f16_add_clamp(acc, ((uint16_t*)bufs[p])[i]);
          for (int p = 0; p < n; p++) ((uint16_t*)bufs[p])[i] = acc;
        } else {
          uint16_t acc = ((uint16_t*)bufs[r])[i];
          for (int p = 0; p < n; p++)
            if (p != r) acc = f32_to_bf16(bf16_to_f32(acc) + bf16_to_f32(((uint16_t*)bufs[p])[i]));
          for (int p = 0; p < n; p++) ((uint16_t*)bufs[p])[i] = acc;
        }
      }
    }
  }
  return used;
}
