// fold.h -- the reference reduce support kernel's per-element fold
// (codegen/templates/reduce.cl:65-69,100-105,120-125; SHIFT_REG and init
// values codegen/ops.py:110-141), shared by the device fold kernel
// (collectives.hip, whole buffers) and the element-granular SMI_Reduce
// (channels.cpp, one element per call on the root).  One source for both:
// IEEE round-to-nearest adds and compares, never contracted
// (-ffp-contract=off), so host and device give the same bits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <limits>
#include <type_traits>

#include "smi.h"

namespace smi {

// include/smi/reduce_operations.h:4-6; integer adds wrap (two's complement)
template <typename T, int OP>
__host__ __device__ __forceinline__ T op_apply(T a, T b) {
    if constexpr (OP == SMI_ADD) {
        if constexpr (std::is_floating_point<T>::value) {
            return a + b;
        } else {
            using U = typename std::make_unsigned<T>::type;
            return (T)(U)((U)a + (U)b);
        }
    } else if constexpr (OP == SMI_MAX) {
        return a > b ? a : b;
    } else {
        return a < b ? a : b;
    }
}

// codegen/ops.py:124-141 SHIFT_REG_INIT (FLT_MIN / DBL_MIN, the smallest
// positive normals, for MAX -- kept as the reference has it)
template <typename T, int OP>
__host__ __device__ __forceinline__ T op_init() {
    if constexpr (OP == SMI_ADD) return (T)0;
    else if constexpr (OP == SMI_MAX) {
        if constexpr (std::is_same<T, float>::value) return 1.17549435e-38f;
        else if constexpr (std::is_same<T, double>::value) return 2.2250738585072014e-308;
        else return std::numeric_limits<T>::min();
    } else {
        if constexpr (std::is_same<T, float>::value) return 3.40282347e+38f;
        else if constexpr (std::is_same<T, double>::value) return 1.7976931348623157e+308;
        else return std::numeric_limits<T>::max();
    }
}

// One element: contributions d[0..n) in rank order (the canonical arrival),
// S rotating slots: q <- [q1 .. q_{S-1}, d_k (+) q0]; result
// ((init (+) q0) (+) q1) ... (+) q_{S-1}.
template <typename T, int S, int OP>
__host__ __device__ __forceinline__ T fold_one(const T *d, int n) {
    T q[S];
    for (int j = 0; j < S; ++j) q[j] = op_init<T, OP>();
    for (int k = 0; k < n; ++k) {
        const T nv = op_apply<T, OP>(d[k], q[0]);
        for (int j = 0; j < S - 1; ++j) q[j] = q[j + 1];
        q[S - 1] = nv;
    }
    T res = op_init<T, OP>();
    for (int j = 0; j < S; ++j) res = op_apply<T, OP>(res, q[j]);
    return res;
}

}  // namespace smi
