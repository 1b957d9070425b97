"""ORACLE (test infrastructure only) — the reference's elementwise reduction functors on the CPU.

Restates /root/reference/src/collectives/device/reduce_kernel.h as numpy operations:
  FuncSum/Prod/Max/Min generic        reduce_kernel.h:23-51     (x+y, x*y, (x<y)?y:x, (x<y)?x:y)
  FuncSum<half>  (sm_80 path)         reduce_kernel.h:244-278   RNE16(x+y) then clamp to [-65504, 65504]
                                                                 (__hmax/__hmin with NaN -> the other operand,
                                                                 so a NaN sum becomes -65504)
  FuncSum<bf16>  (sm_80 path)         reduce_kernel.h:280-303   __hadd2: bf16 RNE of the exact sum
  FuncProd<half>/<bf16>               reduce_kernel.h:305-350   RNE of the exact product, no clamp
  FuncMax/Min<half>                   reduce_kernel.h:352-388   via fmaxf/fminf on the fp32 values
  FuncMax/Min<bf16> (sm_80)           reduce_kernel.h:390-440   __hmax2/__hmin2 (NaN -> other)
  FuncMax/Min<float>/<double>         reduce_kernel.h:442-470   fmaxf/fminf, fmax/fmin
  integer types                        reduce_kernel.h:64-230    two's-complement wrap-around
  FuncPreMulSum / FuncSumPostDiv      reduce_kernel.h:498-687   a sum whose inputs are scaled first
                                                                 (x*scale, one rounding: __hmul/__hmul2/
                                                                 fp32/fp64 multiply, integer wrap) or whose
                                                                 result is divided after (T(x/n), C
                                                                 truncation; integer types only)
  ncclAvg                             enqueue.cc:1388-1454      PreMulSum by 1/n rounded to the type
                                                                 (floats), SumPostDiv by n (integers)
fp16/bf16 sums are formed in fp32 and rounded once to the 16-bit format; for a sum or product
of two p-bit values an fp32 (24-bit) intermediate satisfies q >= 2p+2, so the double rounding is
innocuous and the result equals the correctly rounded value the reference's __hadd2/__hmul2 give.
Third-party pin: cuda_fp16.h / cuda_bf16.h (CUDA >= 11.0) are not in this image; NaN payloads
and the sign of a zero produced by max/min of (+0,-0) are "parity unpinned".
"""
from __future__ import annotations

import numpy as np

SUM, PROD, MAX, MIN, PREMULSUM, SUMPOSTDIV = 0, 1, 2, 3, 4, 5
AVG = 4  # ncclAvg (host op); lowered by avg_op() to PREMULSUM or SUMPOSTDIV

# ncclDataType_t -> (numpy storage dtype, element size, kind)
DTYPES = {
    0: (np.int8, 1, "int"), 1: (np.uint8, 1, "int"), 2: (np.int32, 4, "int"), 3: (np.uint32, 4, "int"),
    4: (np.int64, 8, "int"), 5: (np.uint64, 8, "int"), 6: (np.float16, 2, "f16"),
    7: (np.float32, 4, "f32"), 8: (np.float64, 8, "f64"), 9: (np.uint16, 2, "bf16"),
}
NAMES = {"int8": 0, "uint8": 1, "int32": 2, "uint32": 3, "int64": 4, "uint64": 5,
         "float16": 6, "fp16": 6, "half": 6, "float32": 7, "fp32": 7, "float": 7,
         "float64": 8, "fp64": 8, "double": 8, "bfloat16": 9, "bf16": 9}


def storage(dt: int):
    return DTYPES[dt][0]


def type_size(dt: int) -> int:
    return DTYPES[dt][1]


def bf16_to_f32(u: np.ndarray) -> np.ndarray:
    return (u.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(f: np.ndarray) -> np.ndarray:
    """round-to-nearest-even f32 -> bf16 bits; NaN -> quiet NaN keeping the sign."""
    u = np.ascontiguousarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(f)
    if nan.any():
        r = np.where(nan, ((u >> 16).astype(np.uint16) | np.uint16(0x40)), r)
    return r.astype(np.uint16)


def _clamp_f16(r: np.ndarray) -> np.ndarray:
    r = np.where(np.isnan(r), np.float16(-65504.0), r)
    return np.clip(r, np.float16(-65504.0), np.float16(65504.0)).astype(np.float16)


def apply(op: int, dt: int, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """fn(x, y) with the reference's operand order (x is the first functor argument)."""
    if op in (PREMULSUM, SUMPOSTDIV):   # both reduce with FuncSum (reduce_kernel.h:498-520)
        op = SUM
    kind = DTYPES[dt][2]
    with np.errstate(all="ignore"):
        if kind == "int":
            if op == SUM:
                return (x + y).astype(x.dtype)
            if op == PROD:
                return (x * y).astype(x.dtype)
            if op == MAX:
                return np.where(x < y, y, x)
            return np.where(x < y, x, y)
        if kind in ("f32", "f64"):
            if op == SUM:
                return x + y
            if op == PROD:
                return x * y
            if op == MAX:
                return np.fmax(x, y)
            return np.fmin(x, y)
        if kind == "f16":
            fx, fy = x.astype(np.float32), y.astype(np.float32)
            if op == SUM:
                return _clamp_f16((fx + fy).astype(np.float16))
            if op == PROD:
                return (fx * fy).astype(np.float16)
            if op == MAX:
                return np.fmax(fx, fy).astype(np.float16)
            return np.fmin(fx, fy).astype(np.float16)
        # bf16 stored as uint16 bits
        fx, fy = bf16_to_f32(x), bf16_to_f32(y)
        if op == SUM:
            return f32_to_bf16(fx + fy)
        if op == PROD:
            return f32_to_bf16(fx * fy)
        if op == MAX:
            return f32_to_bf16(np.fmax(fx, fy))
        return f32_to_bf16(np.fmin(fx, fy))


def scalar_bits(dt: int, value) -> int:
    """The 64-bit opArg of a PreMulSum scale: the value's bits in the element type, low bytes."""
    a = from_float(dt, np.array([value], dtype=np.float64)) if DTYPES[dt][2] != "int" else \
        np.array([value]).astype(storage(dt))
    return int.from_bytes(np.ascontiguousarray(a).tobytes().ljust(8, b"\0"), "little")


def avg_op(dt: int, nranks: int):
    """hostToDevRedOp for ncclAvg (enqueue.cc:1403-1431): (device op, opArg).  The scale is
    1.0/n rounded through float for f16/bf16/f32 (__float2half(float(1.0/n)) etc.), 1.0/n for f64."""
    kind = DTYPES[dt][2]
    if kind == "int":
        return SUMPOSTDIV, nranks
    if kind == "f64":
        return PREMULSUM, scalar_bits(dt, 1.0 / nranks)
    return PREMULSUM, scalar_bits(dt, float(np.float32(1.0 / nranks)))


def _scale_of(dt: int, arg: int):
    b = int(arg).to_bytes(8, "little")[:type_size(dt)]
    return np.frombuffer(b, dtype=storage(dt))[0]


def pre_op(op: int, dt: int, x: np.ndarray, arg: int) -> np.ndarray:
    """FuncPreMulSum::preOp: x * scale with one rounding in the element type; identity otherwise."""
    if op != PREMULSUM:
        return x
    kind = DTYPES[dt][2]
    s = _scale_of(dt, arg)
    with np.errstate(all="ignore"):
        if kind == "int":
            return (x * s).astype(x.dtype)
        if kind in ("f32", "f64"):
            return (x * s).astype(x.dtype)
        if kind == "f16":
            return (x.astype(np.float32) * np.float32(s)).astype(np.float16)   # exact in fp32, one RNE
        return f32_to_bf16(bf16_to_f32(x) * bf16_to_f32(np.array([s], np.uint16))[0])


def post_op(op: int, dt: int, x: np.ndarray, arg: int) -> np.ndarray:
    """FuncSumPostDiv::postOp: T(x / n) with C truncation toward zero; identity otherwise."""
    if op != SUMPOSTDIV:
        return x
    n = int(arg)
    xi = x.astype(np.int64) if x.dtype != np.uint64 else x
    if x.dtype == np.uint64:
        return (x // np.uint64(n)).astype(x.dtype)
    q = np.abs(xi) // n * np.sign(xi)
    return q.astype(x.dtype)


def to_float64(dt: int, a: np.ndarray) -> np.ndarray:
    if DTYPES[dt][2] == "bf16":
        return bf16_to_f32(a).astype(np.float64)
    return a.astype(np.float64)


def from_float(dt: int, a: np.ndarray) -> np.ndarray:
    kind = DTYPES[dt][2]
    if kind == "bf16":
        return f32_to_bf16(np.asarray(a, dtype=np.float32))
    return np.asarray(a).astype(storage(dt))


def ulp_distance(dt: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|a-b| in units in the last place of the storage format (monotone integer mapping)."""
    kind = DTYPES[dt][2]
    if kind == "int":
        return np.abs(a.astype(np.int64) - b.astype(np.int64))
    if kind == "f16":
        ia, ib = a.view(np.int16).astype(np.int64), b.view(np.int16).astype(np.int64)
        bits = 16
    elif kind == "bf16":
        ia, ib = a.view(np.int16).astype(np.int64), b.view(np.int16).astype(np.int64)
        bits = 16
    elif kind == "f32":
        ia, ib = a.view(np.int32).astype(np.int64), b.view(np.int32).astype(np.int64)
        bits = 32
    else:
        ia, ib = a.view(np.int64), b.view(np.int64)
        bits = 64
    m = np.int64(1) << np.int64(bits - 1) if bits < 64 else np.int64(-(2 ** 63))

    def key(i):
        if bits == 64:
            return np.where(i < 0, np.int64(-(2 ** 63)) - i, i)
        return np.where(i < 0, -(i & (m - 1)), i)
    return np.abs(key(ia) - key(ib))
