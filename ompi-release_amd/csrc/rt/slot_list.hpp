// slot_list.hpp -- the (MPI_Op, element type) slots that have a GPU kernel, as one list shared by
// the kernel families (the 3-buff table of op_base_functions.c:1460-1543 minus the two 32-byte
// types -- MPI_LONG_DOUBLE_INT and C_LONG_DOUBLE_COMPLEX -- which op/hip's kernels reduce but the
// engine's 16-byte-vector families do not carry: the engine serves those by gather-then-fold).
//
//   for_each_slot([&](auto tag, int op, int type) { using F = typename decltype(tag)::type; ... });
#pragma once

#include "op_functors.hpp"

namespace mi355x {

template <class F> struct SlotTag {
    using type = F;
};

template <template <typename> class OP, class Put> __host__ __device__ inline void for_each_int_slot(Put &&put, int op)
{
    put(SlotTag<OP<int8_t>>{}, op, MI355X_T_INT8);
    put(SlotTag<OP<uint8_t>>{}, op, MI355X_T_UINT8);
    put(SlotTag<OP<int16_t>>{}, op, MI355X_T_INT16);
    put(SlotTag<OP<uint16_t>>{}, op, MI355X_T_UINT16);
    put(SlotTag<OP<int32_t>>{}, op, MI355X_T_INT32);
    put(SlotTag<OP<uint32_t>>{}, op, MI355X_T_UINT32);
    put(SlotTag<OP<int64_t>>{}, op, MI355X_T_INT64);
    put(SlotTag<OP<uint64_t>>{}, op, MI355X_T_UINT64);
}

template <class Put> __host__ __device__ inline void for_each_slot(Put &&put)
{
    for_each_int_slot<OpMax>(put, MI355X_OP_MAX);
    put(SlotTag<OpMax<float>>{}, MI355X_OP_MAX, MI355X_T_FLOAT);
    put(SlotTag<OpMax<double>>{}, MI355X_OP_MAX, MI355X_T_DOUBLE);
    for_each_int_slot<OpMin>(put, MI355X_OP_MIN);
    put(SlotTag<OpMin<float>>{}, MI355X_OP_MIN, MI355X_T_FLOAT);
    put(SlotTag<OpMin<double>>{}, MI355X_OP_MIN, MI355X_T_DOUBLE);
    for_each_int_slot<OpSum>(put, MI355X_OP_SUM);
    put(SlotTag<OpSum<float>>{}, MI355X_OP_SUM, MI355X_T_FLOAT);
    put(SlotTag<OpSum<double>>{}, MI355X_OP_SUM, MI355X_T_DOUBLE);
    put(SlotTag<OpCsum<cf32>>{}, MI355X_OP_SUM, MI355X_T_C_FLOAT_COMPLEX);
    put(SlotTag<OpCsum<cf64>>{}, MI355X_OP_SUM, MI355X_T_C_DOUBLE_COMPLEX);
    for_each_int_slot<OpProd>(put, MI355X_OP_PROD);
    put(SlotTag<OpProd<float>>{}, MI355X_OP_PROD, MI355X_T_FLOAT);
    put(SlotTag<OpProd<double>>{}, MI355X_OP_PROD, MI355X_T_DOUBLE);
    put(SlotTag<OpCprod<cf32>>{}, MI355X_OP_PROD, MI355X_T_C_FLOAT_COMPLEX);
    put(SlotTag<OpCprod<cf64>>{}, MI355X_OP_PROD, MI355X_T_C_DOUBLE_COMPLEX);
    for_each_int_slot<OpLand>(put, MI355X_OP_LAND);
    put(SlotTag<OpLand<uint8_t>>{}, MI355X_OP_LAND, MI355X_T_BOOL);
    for_each_int_slot<OpLor>(put, MI355X_OP_LOR);
    put(SlotTag<OpLor<uint8_t>>{}, MI355X_OP_LOR, MI355X_T_BOOL);
    for_each_int_slot<OpLxor>(put, MI355X_OP_LXOR);
    put(SlotTag<OpLxor<uint8_t>>{}, MI355X_OP_LXOR, MI355X_T_BOOL);
    for_each_int_slot<OpBand>(put, MI355X_OP_BAND);
    put(SlotTag<OpBand<int8_t>>{}, MI355X_OP_BAND, MI355X_T_BYTE);
    for_each_int_slot<OpBor>(put, MI355X_OP_BOR);
    put(SlotTag<OpBor<int8_t>>{}, MI355X_OP_BOR, MI355X_T_BYTE);
    for_each_int_slot<OpBxor>(put, MI355X_OP_BXOR);
    put(SlotTag<OpBxor<int8_t>>{}, MI355X_OP_BXOR, MI355X_T_BYTE);
    put(SlotTag<OpLoc<p_float_int, true>>{}, MI355X_OP_MAXLOC, MI355X_T_FLOAT_INT);
    put(SlotTag<OpLoc<p_double_int, true>>{}, MI355X_OP_MAXLOC, MI355X_T_DOUBLE_INT);
    put(SlotTag<OpLoc<p_long_int, true>>{}, MI355X_OP_MAXLOC, MI355X_T_LONG_INT);
    put(SlotTag<OpLoc<p_2int, true>>{}, MI355X_OP_MAXLOC, MI355X_T_2INT);
    put(SlotTag<OpLoc<p_short_int, true>>{}, MI355X_OP_MAXLOC, MI355X_T_SHORT_INT);
    put(SlotTag<OpLoc<p_float_int, false>>{}, MI355X_OP_MINLOC, MI355X_T_FLOAT_INT);
    put(SlotTag<OpLoc<p_double_int, false>>{}, MI355X_OP_MINLOC, MI355X_T_DOUBLE_INT);
    put(SlotTag<OpLoc<p_long_int, false>>{}, MI355X_OP_MINLOC, MI355X_T_LONG_INT);
    put(SlotTag<OpLoc<p_2int, false>>{}, MI355X_OP_MINLOC, MI355X_T_2INT);
    put(SlotTag<OpLoc<p_short_int, false>>{}, MI355X_OP_MINLOC, MI355X_T_SHORT_INT);
    // x87 long double MAX/MIN: compare-and-select on the 80-bit encoding; SUM/PROD: the x87 add
    // and multiply in integer arithmetic (op_functors.hpp, f80_arith.hpp)
    put(SlotTag<OpMax<f80>>{}, MI355X_OP_MAX, MI355X_T_LONG_DOUBLE);
    put(SlotTag<OpMin<f80>>{}, MI355X_OP_MIN, MI355X_T_LONG_DOUBLE);
    put(SlotTag<OpSum<f80>>{}, MI355X_OP_SUM, MI355X_T_LONG_DOUBLE);
    put(SlotTag<OpProd<f80>>{}, MI355X_OP_PROD, MI355X_T_LONG_DOUBLE);
}

} // namespace mi355x
