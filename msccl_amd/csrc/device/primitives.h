// Memory-access helpers and elementwise reduction functors for the gfx950 MSCCL kernels.
//
// Reduction semantics follow the reference functors (collectives/device/reduce_kernel.h):
//   Sum/Prod/Max/Min (23-51), FuncSum<half> with the sm_80 +-65504 clamp (244-278),
//   FuncSum<bf16> = bf16 RNE of the exact sum (280-303), half/bf16 Prod/Max/Min (305-440),
//   float/double Max/Min = fmax/fmin (442-470), integer types wrap (64-230).
// fp16 is added with v_pk_add_f16 (correctly rounded) and clamped with v_pk_max/min_f16;
// bf16 is widened to fp32, added and rounded once with v_cvt_pk_bf16_f32 (RNE): for a sum of
// two 8-bit-significand values an fp32 intermediate makes the double rounding innocuous.
//
// Cache policy (gfx950 CPol bits: sc0=1, nt=2, sc1=16):
//   local buffers (user input/output/scratch) are read and written with sc1 (device scope)
//   so that a hand-off between workgroups through a dependency flag needs no L2/L1
//   maintenance fence (MI355X guide, inter-workgroup visibility, "sc1 stores + sc1 loads");
//   FIFOs live in uncached fine-grained memory of the receiver and are accessed sc0|sc1.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "devcomm.h"

namespace msccl {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

constexpr int kAuxLocal = 16;   // sc1
constexpr int kAuxFifo = 17;    // sc0 | sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t makeRsrc(const void* p) {
  uint64_t a = (uint64_t)p;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}

// Wave-uniform values read from LDS land in VGPRs; readfirstlane moves them to SGPRs so the
// interpreter state stays out of the vector register budget of the hot loops.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// (readfirstlane returns int: both halves go through uint32_t, or a low half with bit 31 set
// would sign-extend over the high half)
__device__ __forceinline__ uint64_t uni(uint64_t x) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
  return ((uint64_t)hi << 32) | lo;
}

// Kernel-argument values a prologue needs, held in SGPRs from here on: without it the compiler
// sinks each scalar load into the branch that uses it, and every lane group's load chain starts
// with its own kernel-argument round trip (three in a row in the fold kernel).  An empty asm
// statement with SGPR inputs: no instruction, only the order of issue.
template <class A>
__device__ __forceinline__ void pinArg(const A& a) {
  asm volatile("" ::"s"(a));
}
template <class... A>
__device__ __forceinline__ void pinArgs(const A&... a) {
  (pinArg(a), ...);
}

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
template <int AUX>
__device__ __forceinline__ u32x3 ld12(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void st12(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x3 v) {
  __builtin_amdgcn_raw_buffer_store_b96(v, r, off, 0, AUX);
}

template <int AUX>
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

// Element loads/stores for tails and unaligned buffers.
template <typename T>
__device__ __forceinline__ T ldElem(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (sizeof(T) == 1) {
    uint8_t v = __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, kAuxLocal);
    return __builtin_bit_cast(T, v);
  } else if constexpr (sizeof(T) == 2) {
    uint16_t v = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, kAuxLocal);
    return __builtin_bit_cast(T, v);
  } else if constexpr (sizeof(T) == 4) {
    uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kAuxLocal);
    return __builtin_bit_cast(T, v);
  } else {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxLocal);
    return __builtin_bit_cast(T, v);
  }
}
template <typename T>
__device__ __forceinline__ void stElem(__amdgpu_buffer_rsrc_t r, uint32_t off, T x) {
  if constexpr (sizeof(T) == 1) {
    __builtin_amdgcn_raw_buffer_store_b8(__builtin_bit_cast(uint8_t, x), r, off, 0, kAuxLocal);
  } else if constexpr (sizeof(T) == 2) {
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, x), r, off, 0, kAuxLocal);
  } else if constexpr (sizeof(T) == 4) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), r, off, 0, kAuxLocal);
  } else {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, x), r, off, 0, kAuxLocal);
  }
}

// Two FIFO lines polled together: both loads in flight, one wait (form (i) of the guide's
// inline-asm rules: the loads and their s_waitcnt in one statement, early-clobber outputs).
__device__ __forceinline__ void ldLines2(const void* a, const void* b, u32x4& x, u32x4& y) {
  asm volatile(
      "global_load_dwordx4 %0, %2, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %3, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x), "=&v"(y)
      : "v"(a), "v"(b)
      : "memory");
}
// Four FIFO lines in flight, one wait.
__device__ __forceinline__ void ldLines4(const void* const* p, u32x4* x) {
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %5, off sc0 sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc0 sc1\n\t"
      "global_load_dwordx4 %3, %7, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
      : "memory");
}
// Eight FIFO lines (four packs) in flight, one wait.
__device__ __forceinline__ void ldLines8(const void* const* p, u32x4* x) {
  asm volatile(
      "global_load_dwordx4 %0, %8, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %9, off sc0 sc1\n\t"
      "global_load_dwordx4 %2, %10, off sc0 sc1\n\t"
      "global_load_dwordx4 %3, %11, off sc0 sc1\n\t"
      "global_load_dwordx4 %4, %12, off sc0 sc1\n\t"
      "global_load_dwordx4 %5, %13, off sc0 sc1\n\t"
      "global_load_dwordx4 %6, %14, off sc0 sc1\n\t"
      "global_load_dwordx4 %7, %15, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
// Sixteen FIFO lines (the flat tree's fold: two lines of 8 peers) in flight, one wait.  Every
// address is a VGPR pair: no SGPR operand in inline asm, whose "VALU writes SGPR -> VMEM reads it"
// wait states the compiler's hazard recognizer does not insert for asm (a readfirstlane'd slot
// base used as a global_ saddr right after it read a stale base and faulted, timing-dependent).
__device__ __forceinline__ void ldLines16(const void* const* p, u32x4* x) {
  asm volatile(
      "global_load_dwordx4 %0, %16, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %17, off sc0 sc1\n\t"
      "global_load_dwordx4 %2, %18, off sc0 sc1\n\t"
      "global_load_dwordx4 %3, %19, off sc0 sc1\n\t"
      "global_load_dwordx4 %4, %20, off sc0 sc1\n\t"
      "global_load_dwordx4 %5, %21, off sc0 sc1\n\t"
      "global_load_dwordx4 %6, %22, off sc0 sc1\n\t"
      "global_load_dwordx4 %7, %23, off sc0 sc1\n\t"
      "global_load_dwordx4 %8, %24, off sc0 sc1\n\t"
      "global_load_dwordx4 %9, %25, off sc0 sc1\n\t"
      "global_load_dwordx4 %10, %26, off sc0 sc1\n\t"
      "global_load_dwordx4 %11, %27, off sc0 sc1\n\t"
      "global_load_dwordx4 %12, %28, off sc0 sc1\n\t"
      "global_load_dwordx4 %13, %29, off sc0 sc1\n\t"
      "global_load_dwordx4 %14, %30, off sc0 sc1\n\t"
      "global_load_dwordx4 %15, %31, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(x[4]), "=&v"(x[5]), "=&v"(x[6]), "=&v"(x[7]),
        "=&v"(x[8]), "=&v"(x[9]), "=&v"(x[10]), "=&v"(x[11]), "=&v"(x[12]), "=&v"(x[13]), "=&v"(x[14]), "=&v"(x[15])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]),
        "v"(p[8]), "v"(p[9]), "v"(p[10]), "v"(p[11]), "v"(p[12]), "v"(p[13]), "v"(p[14]), "v"(p[15])
      : "memory");
}
// The fold kernels' batch: two lines of each of G peers in flight, one wait.  The array sizes are
// part of the type, so a batch whose arrays do not hold exactly 2 G lines does not compile (a
// variant that passed 8-entry arrays to ldLines16 read past them and faulted).
template <int G>
__device__ __forceinline__ void ldLinesPeers(const void* const (&p)[2 * G], u32x4 (&x)[2 * G]) {
  static_assert(G == 4 || G == 8, "batches of 4 or 8 peers");
  if constexpr (G == 8) ldLines16(p, x);
  else ldLines8(p, x);
}
__device__ __forceinline__ void ldLine1(const void* a, u32x4& x) {
  asm volatile(
      "global_load_dwordx4 %0, %1, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(x)
      : "v"(a)
      : "memory");
}

// Flag / credit words.  The pointers come from LDS copies of the connection records, so the
// compiler cannot prove their address space and would emit flat_ accesses; the guide's hand-off
// forms are stated for global_/buffer_ instructions (never flat_), so every word access is made
// explicitly global (address space 1).
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ uint64_t atomicLoadSys(const uint64_t* p) {
  return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void atomicStoreSys(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t atomicLoadAgent(const uint64_t* p) {
  return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void atomicStoreAgent(uint64_t* p, uint64_t v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t atomicLoadSys32(const volatile uint32_t* p) {
  return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void atomicStoreSys32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drainStores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------------------------
// Elementwise functors.  fn(x, y) keeps the reference's operand order.
// kPreMulSum / kSumPostDiv are the reference's device ops for ncclAvg and user PreMulSum ops
// (reduce_kernel.h:498-560, enqueue.cc:1388-1454): a sum whose inputs are scaled before (preOp)
// or whose result is divided after (postOp).  They only run in the ring fallback, as in the
// reference, where MSCCL admits Sum/Prod/Max/Min only (tuning.cc:345).
enum RedOp { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kPreMulSum = 4, kSumPostDiv = 5 };
constexpr int baseOp(int op) { return op >= kPreMulSum ? kSum : op; }

template <typename T> struct IsHalf { static constexpr bool v = false; };
template <> struct IsHalf<_Float16> { static constexpr bool v = true; };

struct Bf16 { uint16_t bits; };  // bf16 storage type

template <typename T, int OP>
struct Fn {
  __device__ __forceinline__ static T elem(T x, T y) {
    using U = typename std::make_unsigned<T>::type;  // two's-complement wrap, no signed-overflow UB
    constexpr int B = baseOp(OP);
    if constexpr (B == kSum) return (T)(U)((U)x + (U)y);
    else if constexpr (B == kProd) return (T)(U)((U)x * (U)y);
    else if constexpr (B == kMax) return (x < y) ? y : x;
    else return (x < y) ? x : y;
  }
  __device__ __forceinline__ static u32x4 pack(u32x4 a, u32x4 b) {
    constexpr int N = 16 / sizeof(T);
    T xa[N], xb[N];
    __builtin_memcpy(xa, &a, 16);
    __builtin_memcpy(xb, &b, 16);
#pragma unroll
    for (int i = 0; i < N; i++) xa[i] = elem(xa[i], xb[i]);
    u32x4 r;
    __builtin_memcpy(&r, xa, 16);
    return r;
  }
};

template <int OP>
struct Fn<float, OP> {
  __device__ __forceinline__ static float elem(float x, float y) {
    constexpr int B = baseOp(OP);
    if constexpr (B == kSum) return x + y;
    else if constexpr (B == kProd) return x * y;
    else if constexpr (B == kMax) return __builtin_fmaxf(x, y);
    else return __builtin_fminf(x, y);
  }
  __device__ __forceinline__ static uint32_t e1(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, elem(__builtin_bit_cast(float, a), __builtin_bit_cast(float, b)));
  }
  __device__ __forceinline__ static u32x4 pack(u32x4 a, u32x4 b) {
    return (u32x4){e1(a.x, b.x), e1(a.y, b.y), e1(a.z, b.z), e1(a.w, b.w)};
  }
};

template <int OP>
struct Fn<double, OP> {
  __device__ __forceinline__ static double elem(double x, double y) {
    constexpr int B = baseOp(OP);
    if constexpr (B == kSum) return x + y;
    else if constexpr (B == kProd) return x * y;
    else if constexpr (B == kMax) return __builtin_fmax(x, y);
    else return __builtin_fmin(x, y);
  }
  __device__ __forceinline__ static u32x4 pack(u32x4 a, u32x4 b) {
    double xa[2], xb[2];
    __builtin_memcpy(xa, &a, 16);
    __builtin_memcpy(xb, &b, 16);
    xa[0] = elem(xa[0], xb[0]);
    xa[1] = elem(xa[1], xb[1]);
    u32x4 r;
    __builtin_memcpy(&r, xa, 16);
    return r;
  }
};

template <int OP>
struct Fn<_Float16, OP> {
  __device__ __forceinline__ static f16x2 op2(f16x2 x, f16x2 y) {
    constexpr int B = baseOp(OP);
    if constexpr (B == kSum) {
      f16x2 r = x + y;  // v_pk_add_f16, RNE
      r = __builtin_elementwise_max(r, (f16x2){(_Float16)-65504.0f, (_Float16)-65504.0f});
      r = __builtin_elementwise_min(r, (f16x2){(_Float16)65504.0f, (_Float16)65504.0f});
      return r;
    } else if constexpr (B == kProd) {
      return x * y;
    } else {
      f32x2 fx = __builtin_convertvector(x, f32x2), fy = __builtin_convertvector(y, f32x2);
      f32x2 m;
      if constexpr (B == kMax) m = (f32x2){__builtin_fmaxf(fx[0], fy[0]), __builtin_fmaxf(fx[1], fy[1])};
      else m = (f32x2){__builtin_fminf(fx[0], fy[0]), __builtin_fminf(fx[1], fy[1])};
      return __builtin_convertvector(m, f16x2);
    }
  }
  __device__ __forceinline__ static _Float16 elem(_Float16 x, _Float16 y) {
    f16x2 r = op2((f16x2){x, x}, (f16x2){y, y});
    return r[0];
  }
  __device__ __forceinline__ static uint32_t e1(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, op2(__builtin_bit_cast(f16x2, a), __builtin_bit_cast(f16x2, b)));
  }
  __device__ __forceinline__ static u32x4 pack(u32x4 a, u32x4 b) {
    return (u32x4){e1(a.x, b.x), e1(a.y, b.y), e1(a.z, b.z), e1(a.w, b.w)};
  }
};

template <int OP>
struct Fn<Bf16, OP> {
  __device__ __forceinline__ static bf16x2 op2(bf16x2 x, bf16x2 y) {
    f32x2 fx = __builtin_convertvector(x, f32x2), fy = __builtin_convertvector(y, f32x2);
    f32x2 r;
    constexpr int B = baseOp(OP);
    if constexpr (B == kSum) r = fx + fy;
    else if constexpr (B == kProd) r = fx * fy;
    else if constexpr (B == kMax) r = (f32x2){__builtin_fmaxf(fx[0], fy[0]), __builtin_fmaxf(fx[1], fy[1])};
    else r = (f32x2){__builtin_fminf(fx[0], fy[0]), __builtin_fminf(fx[1], fy[1])};
    return __builtin_convertvector(r, bf16x2);  // v_cvt_pk_bf16_f32 (RNE)
  }
  __device__ __forceinline__ static Bf16 elem(Bf16 x, Bf16 y) {
    uint32_t ux = x.bits * 0x10001u, uy = y.bits * 0x10001u;
    bf16x2 r = op2(__builtin_bit_cast(bf16x2, ux), __builtin_bit_cast(bf16x2, uy));
    Bf16 o;
    o.bits = (uint16_t)__builtin_bit_cast(uint32_t, r);
    return o;
  }
  __device__ __forceinline__ static uint32_t e1(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, op2(__builtin_bit_cast(bf16x2, a), __builtin_bit_cast(bf16x2, b)));
  }
  __device__ __forceinline__ static u32x4 pack(u32x4 a, u32x4 b) {
    return (u32x4){e1(a.x, b.x), e1(a.y, b.y), e1(a.z, b.z), e1(a.w, b.w)};
  }
};

// ---------------------------------------------------------------------------------------------
// preOp / postOp of kPreMulSum and kSumPostDiv (reduce_kernel.h:498-687); identity otherwise.
// The scalar travels as the reference's 64-bit opArg: the scale's bits in the low bytes
// (PreMulSum) or the rank count (SumPostDiv).
template <typename T, int OP>
struct PrePost {
  static constexpr bool kPre = false, kPost = false;
  __device__ __forceinline__ static u32x4 pre(u32x4 v, uint64_t) { return v; }
  __device__ __forceinline__ static u32x4 post(u32x4 v, uint64_t) { return v; }
};

template <typename T>
__device__ __forceinline__ T scaleElem(T x, uint64_t arg) {
  T s;
  __builtin_memcpy(&s, &arg, sizeof(T));
  if constexpr (std::is_same<T, float>::value || std::is_same<T, double>::value) {
    return x * s;
  } else if constexpr (std::is_same<T, _Float16>::value) {
    return x * s;                                        // v_mul_f16 / __hmul: one rounding
  } else if constexpr (std::is_same<T, Bf16>::value) {
    uint32_t fx = (uint32_t)x.bits << 16, fs = (uint32_t)s.bits << 16;
    const float p = __builtin_bit_cast(float, fx) * __builtin_bit_cast(float, fs);  // exact in fp32
    const bf16x2 r = __builtin_convertvector((f32x2){p, p}, bf16x2);              // RNE to bf16
    Bf16 o;
    o.bits = (uint16_t)__builtin_bit_cast(uint32_t, r);
    return o;
  } else {
    using U = typename std::make_unsigned<T>::type;     // FuncPreMulSum<int>: x * scale, wrapping
    return (T)(U)((U)x * (U)s);
  }
}

template <typename T>
struct PrePost<T, kPreMulSum> {
  static constexpr bool kPre = true, kPost = false;
  __device__ __forceinline__ static u32x4 pre(u32x4 v, uint64_t arg) {
    constexpr int N = 16 / sizeof(T);
    T x[N];
    __builtin_memcpy(x, &v, 16);
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = scaleElem<T>(x[i], arg);
    __builtin_memcpy(&v, x, 16);
    return v;
  }
  __device__ __forceinline__ static u32x4 post(u32x4 v, uint64_t) { return v; }
};

template <typename T>
struct PrePost<T, kSumPostDiv> {  // integral types only (reduce_kernel.h:498-517)
  static constexpr bool kPre = false, kPost = true;
  __device__ __forceinline__ static u32x4 pre(u32x4 v, uint64_t) { return v; }
  __device__ __forceinline__ static u32x4 post(u32x4 v, uint64_t arg) {
    constexpr int N = 16 / sizeof(T);
    const int n = (int)arg;
    T x[N];
    __builtin_memcpy(x, &v, 16);
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = T(x[i] / n);       // T(x/n) with int n, as the reference
    __builtin_memcpy(&v, x, 16);
    return v;
  }
};

}  // namespace msccl
