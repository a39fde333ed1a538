/*
 * op_oracle.c -- CPU restatement of the Open MPI 1.8.5 intrinsic reduction loops.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Restates, per (op, type):
 *   2-buff  `out op= in` / `out = f(out, in)`           op_base_functions.c:39-72
 *   2-buff  MAXLOC/MINLOC pair rule                      op_base_functions.c:81-103
 *   3-buff  `out = in1 op in2` / `out = f(in1, in2)`     op_base_functions.c:606-644
 *   3-buff  MAXLOC/MINLOC pair rule                      op_base_functions.c:661-683
 *   which slots exist (Fortran disabled)                 op_base_functions.c:1192-1361,1373-1543
 * Operand roles are kept exactly: in every 2-buff expression `o` is the inout (target) element
 * and `a` the in (source) element; in every 3-buff expression `o` is in1 and `a` is in2.  This
 * matters for MAX/MIN with NaN or signed zeros (`(o > a) ? o : a` selects an operand), for
 * complex PROD (GCC lowers `o * a` to __mulsc3/__muldc3/__mulxc3(o, a)), and for MAXLOC ties.
 * Build flags match the reference (-O3 -finline-functions -fno-strict-aliasing,
 * config/opal_setup_cc.m4:185-213,300-313) so the CPU baseline is a like-for-like loop.
 */
#include "oracle.h"

#include <complex.h>
#include <pthread.h>
#include <stdbool.h>
#include <string.h>

/* pair types, laid out as the C structs of op_base_functions.c:539-555 */
typedef struct { float v; int k; } pr_float_int;
typedef struct { double v; int k; } pr_double_int;
typedef struct { long v; int k; } pr_long_int;
typedef struct { int v; int k; } pr_2int;
typedef struct { short v; int k; } pr_short_int;
typedef struct { long double v; int k; } pr_long_double_int;

typedef void (*fn2_t)(const void *in, void *inout, size_t n);
typedef void (*fn3_t)(const void *in1, const void *in2, void *out, size_t n);

/* One macro emits both the 2-buff and 3-buff loop for an elementwise rule EXPR(o, a). */
#define ELEMWISE(TAG, T, EXPR)                                                         \
    static void o2_##TAG(const void *vin, void *vio, size_t n)                         \
    {                                                                                  \
        const T *src = (const T *)vin;                                                 \
        T *dst = (T *)vio;                                                             \
        for (size_t i = 0; i < n; ++i) {                                               \
            T o = dst[i], a = src[i];                                                  \
            dst[i] = (T)(EXPR);                                                        \
        }                                                                              \
    }                                                                                  \
    static void o3_##TAG(const void *v1, const void *v2, void *vo, size_t n)           \
    {                                                                                  \
        const T *restrict s1 = (const T *)v1;                                          \
        const T *restrict s2 = (const T *)v2;                                          \
        T *restrict d = (T *)vo;                                                       \
        for (size_t i = 0; i < n; ++i) {                                               \
            T o = s1[i], a = s2[i];                                                    \
            d[i] = (T)(EXPR);                                                          \
        }                                                                              \
    }

/* MAXLOC / MINLOC.  CMP is `>` (maxloc) or `<` (minloc).
 * 2-buff (op_base_functions.c:87-103): take `in` when in.v CMP out.v; on equal values keep
 *   out.v and set k = min(out.k, in.k); otherwise leave out untouched.
 * 3-buff (op_base_functions.c:661-683): in1 when in1.v CMP in2.v; on equal values v = in1.v and
 *   k = min; otherwise in2.  Only the v and k members are written (padding left as is). */
#define PAIRWISE(TAG, PT, CMP)                                                         \
    static void o2_##TAG(const void *vin, void *vio, size_t n)                         \
    {                                                                                  \
        const PT *src = (const PT *)vin;                                               \
        PT *dst = (PT *)vio;                                                           \
        for (size_t i = 0; i < n; ++i) {                                               \
            if (src[i].v CMP dst[i].v) {                                               \
                dst[i].v = src[i].v;                                                   \
                dst[i].k = src[i].k;                                                   \
            } else if (src[i].v == dst[i].v) {                                         \
                if (src[i].k < dst[i].k) dst[i].k = src[i].k;                          \
            }                                                                          \
        }                                                                              \
    }                                                                                  \
    static void o3_##TAG(const void *v1, const void *v2, void *vo, size_t n)           \
    {                                                                                  \
        const PT *restrict s1 = (const PT *)v1;                                        \
        const PT *restrict s2 = (const PT *)v2;                                        \
        PT *restrict d = (PT *)vo;                                                     \
        for (size_t i = 0; i < n; ++i) {                                               \
            if (s1[i].v CMP s2[i].v) {                                                 \
                d[i].v = s1[i].v;                                                      \
                d[i].k = s1[i].k;                                                      \
            } else if (s1[i].v == s2[i].v) {                                           \
                d[i].v = s1[i].v;                                                      \
                d[i].k = (s2[i].k < s1[i].k) ? s2[i].k : s1[i].k;                      \
            } else {                                                                   \
                d[i].v = s2[i].v;                                                      \
                d[i].k = s2[i].k;                                                      \
            }                                                                          \
        }                                                                              \
    }

/* rule expressions (o = out/in1, a = in/in2) -- op_base_functions.c:108-533 */
#define R_MAX  ((o) > (a) ? (o) : (a))
#define R_MIN  ((o) < (a) ? (o) : (a))
#define R_SUM  ((o) + (a))
#define R_PROD ((o) * (a))
#define R_LAND ((o) && (a))
#define R_LOR  ((o) || (a))
#define R_LXOR (((o) ? 1 : 0) ^ ((a) ? 1 : 0))
#define R_BAND ((o) & (a))
#define R_BOR  ((o) | (a))
#define R_BXOR ((o) ^ (a))

/* C integer group (op_base_functions.c:1192-1200): every op except the LOC pair ops */
#define INT_GROUP(OPN, RULE)                       \
    ELEMWISE(OPN##_i8, int8_t, RULE)               \
    ELEMWISE(OPN##_u8, uint8_t, RULE)              \
    ELEMWISE(OPN##_i16, int16_t, RULE)             \
    ELEMWISE(OPN##_u16, uint16_t, RULE)            \
    ELEMWISE(OPN##_i32, int32_t, RULE)             \
    ELEMWISE(OPN##_u32, uint32_t, RULE)            \
    ELEMWISE(OPN##_i64, int64_t, RULE)             \
    ELEMWISE(OPN##_u64, uint64_t, RULE)

/* Signed-overflow note: for SUM/PROD the reference loops rely on gcc's two's-complement
 * code generation (UB in ISO C, wraps on x86-64); the oracle does the same arithmetic in the
 * same width, so the bits agree. */
INT_GROUP(max, R_MAX)
INT_GROUP(min, R_MIN)
INT_GROUP(sum, R_SUM)
INT_GROUP(prod, R_PROD)
INT_GROUP(land, R_LAND)
INT_GROUP(lor, R_LOR)
INT_GROUP(lxor, R_LXOR)
INT_GROUP(band, R_BAND)
INT_GROUP(bor, R_BOR)
INT_GROUP(bxor, R_BXOR)

/* floating point group (op_base_functions.c:1295-1300) */
#define FP_GROUP(OPN, RULE)                        \
    ELEMWISE(OPN##_f32, float, RULE)               \
    ELEMWISE(OPN##_f64, double, RULE)              \
    ELEMWISE(OPN##_f80, long double, RULE)
FP_GROUP(max, R_MAX)
FP_GROUP(min, R_MIN)
FP_GROUP(sum, R_SUM)
FP_GROUP(prod, R_PROD)

/* complex group, SUM/PROD only (op_base_functions.c:1321-1324) */
ELEMWISE(sum_c32, float _Complex, R_SUM)
ELEMWISE(sum_c64, double _Complex, R_SUM)
ELEMWISE(sum_c80, long double _Complex, R_SUM)
ELEMWISE(prod_c32, float _Complex, R_PROD)
ELEMWISE(prod_c64, double _Complex, R_PROD)
ELEMWISE(prod_c80, long double _Complex, R_PROD)

/* C bool, logical ops only (op_base_functions.c:1311-1313) */
ELEMWISE(land_bool, bool, R_LAND)
ELEMWISE(lor_bool, bool, R_LOR)
ELEMWISE(lxor_bool, bool, R_LXOR)

/* MPI_BYTE (`char`), bitwise ops only (op_base_functions.c:1328-1329) */
ELEMWISE(band_byte, char, R_BAND)
ELEMWISE(bor_byte, char, R_BOR)
ELEMWISE(bxor_byte, char, R_BXOR)

/* pair types (op_base_functions.c:1352-1361) */
#define LOC_GROUP(OPN, CMP)                                  \
    PAIRWISE(OPN##_float_int, pr_float_int, CMP)             \
    PAIRWISE(OPN##_double_int, pr_double_int, CMP)           \
    PAIRWISE(OPN##_long_int, pr_long_int, CMP)               \
    PAIRWISE(OPN##_2int, pr_2int, CMP)                       \
    PAIRWISE(OPN##_short_int, pr_short_int, CMP)             \
    PAIRWISE(OPN##_long_double_int, pr_long_double_int, CMP)
LOC_GROUP(maxloc, >)
LOC_GROUP(minloc, <)

/* ------------------------------------------------------------------ tables */
static fn2_t T2[MI355X_OP_MAX_][MI355X_T_MAX];
static fn3_t T3[MI355X_OP_MAX_][MI355X_T_MAX];
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

#define SET(OP, TY, TAG) do { T2[OP][TY] = o2_##TAG; T3[OP][TY] = o3_##TAG; } while (0)
#define SET_INTS(OP, OPN)                          \
    do {                                           \
        SET(OP, MI355X_T_INT8, OPN##_i8);          \
        SET(OP, MI355X_T_UINT8, OPN##_u8);         \
        SET(OP, MI355X_T_INT16, OPN##_i16);        \
        SET(OP, MI355X_T_UINT16, OPN##_u16);       \
        SET(OP, MI355X_T_INT32, OPN##_i32);        \
        SET(OP, MI355X_T_UINT32, OPN##_u32);       \
        SET(OP, MI355X_T_INT64, OPN##_i64);        \
        SET(OP, MI355X_T_UINT64, OPN##_u64);       \
    } while (0)
#define SET_FPS(OP, OPN)                           \
    do {                                           \
        SET(OP, MI355X_T_FLOAT, OPN##_f32);        \
        SET(OP, MI355X_T_DOUBLE, OPN##_f64);       \
        SET(OP, MI355X_T_LONG_DOUBLE, OPN##_f80);  \
    } while (0)
#define SET_LOCS(OP, OPN)                                        \
    do {                                                         \
        SET(OP, MI355X_T_FLOAT_INT, OPN##_float_int);            \
        SET(OP, MI355X_T_DOUBLE_INT, OPN##_double_int);          \
        SET(OP, MI355X_T_LONG_INT, OPN##_long_int);              \
        SET(OP, MI355X_T_2INT, OPN##_2int);                      \
        SET(OP, MI355X_T_SHORT_INT, OPN##_short_int);            \
        SET(OP, MI355X_T_LONG_DOUBLE_INT, OPN##_long_double_int);\
    } while (0)

static void build_tables(void)
{
    SET_INTS(MI355X_OP_MAX, max);   SET_FPS(MI355X_OP_MAX, max);
    SET_INTS(MI355X_OP_MIN, min);   SET_FPS(MI355X_OP_MIN, min);
    SET_INTS(MI355X_OP_SUM, sum);   SET_FPS(MI355X_OP_SUM, sum);
    SET(MI355X_OP_SUM, MI355X_T_C_FLOAT_COMPLEX, sum_c32);
    SET(MI355X_OP_SUM, MI355X_T_C_DOUBLE_COMPLEX, sum_c64);
    SET(MI355X_OP_SUM, MI355X_T_C_LONG_DOUBLE_COMPLEX, sum_c80);
    SET_INTS(MI355X_OP_PROD, prod); SET_FPS(MI355X_OP_PROD, prod);
    SET(MI355X_OP_PROD, MI355X_T_C_FLOAT_COMPLEX, prod_c32);
    SET(MI355X_OP_PROD, MI355X_T_C_DOUBLE_COMPLEX, prod_c64);
    SET(MI355X_OP_PROD, MI355X_T_C_LONG_DOUBLE_COMPLEX, prod_c80);
    SET_INTS(MI355X_OP_LAND, land); SET(MI355X_OP_LAND, MI355X_T_BOOL, land_bool);
    SET_INTS(MI355X_OP_LOR, lor);   SET(MI355X_OP_LOR, MI355X_T_BOOL, lor_bool);
    SET_INTS(MI355X_OP_LXOR, lxor); SET(MI355X_OP_LXOR, MI355X_T_BOOL, lxor_bool);
    SET_INTS(MI355X_OP_BAND, band); SET(MI355X_OP_BAND, MI355X_T_BYTE, band_byte);
    SET_INTS(MI355X_OP_BOR, bor);   SET(MI355X_OP_BOR, MI355X_T_BYTE, bor_byte);
    SET_INTS(MI355X_OP_BXOR, bxor); SET(MI355X_OP_BXOR, MI355X_T_BYTE, bxor_byte);
    SET_LOCS(MI355X_OP_MAXLOC, maxloc);
    SET_LOCS(MI355X_OP_MINLOC, minloc);
}

static void ensure_tables(void) { pthread_once(&tables_once, build_tables); }

size_t oracle_type_size(int type)
{
    switch (type) {
    case MI355X_T_INT8: case MI355X_T_UINT8: case MI355X_T_BOOL: case MI355X_T_BYTE: return 1;
    case MI355X_T_INT16: case MI355X_T_UINT16: return 2;
    case MI355X_T_INT32: case MI355X_T_UINT32: case MI355X_T_FLOAT: return 4;
    case MI355X_T_INT64: case MI355X_T_UINT64: case MI355X_T_DOUBLE: return 8;
    case MI355X_T_LONG_DOUBLE: return sizeof(long double);
    case MI355X_T_C_FLOAT_COMPLEX: return sizeof(float _Complex);
    case MI355X_T_C_DOUBLE_COMPLEX: return sizeof(double _Complex);
    case MI355X_T_C_LONG_DOUBLE_COMPLEX: return sizeof(long double _Complex);
    case MI355X_T_FLOAT_INT: return sizeof(pr_float_int);
    case MI355X_T_DOUBLE_INT: return sizeof(pr_double_int);
    case MI355X_T_LONG_INT: return sizeof(pr_long_int);
    case MI355X_T_2INT: return sizeof(pr_2int);
    case MI355X_T_SHORT_INT: return sizeof(pr_short_int);
    case MI355X_T_LONG_DOUBLE_INT: return sizeof(pr_long_double_int);
    default: return 0;
    }
}

int oracle_has_op(int op, int type)
{
    if (op < 0 || op >= MI355X_OP_MAX_ || type < 0 || type >= MI355X_T_MAX) return 0;
    ensure_tables();
    return T2[op][type] != NULL;
}

int oracle_op_2buff(int op, int type, const void *in, void *inout, size_t count)
{
    if (!oracle_has_op(op, type)) return MI355X_ERR_UNSUPPORTED;
    T2[op][type](in, inout, count);
    return MI355X_SUCCESS;
}

int oracle_op_3buff(int op, int type, const void *in1, const void *in2, void *out, size_t count)
{
    if (!oracle_has_op(op, type)) return MI355X_ERR_UNSUPPORTED;
    T3[op][type](in1, in2, out, count);
    return MI355X_SUCCESS;
}

struct mt_slice { fn3_t f; const char *a, *b; char *o; size_t n; };
static void *mt_run(void *p)
{
    struct mt_slice *s = (struct mt_slice *)p;
    s->f(s->a, s->b, s->o, s->n);
    return NULL;
}

int oracle_op_3buff_mt(int op, int type, const void *in1, const void *in2, void *out,
                       size_t count, int nthreads)
{
    if (!oracle_has_op(op, type)) return MI355X_ERR_UNSUPPORTED;
    if (nthreads <= 1) return oracle_op_3buff(op, type, in1, in2, out, count);
    if (nthreads > 256) nthreads = 256;
    size_t esz = oracle_type_size(type);
    pthread_t th[256];
    struct mt_slice sl[256];
    size_t per = count / (size_t)nthreads, rem = count % (size_t)nthreads, off = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t n = per + ((size_t)t < rem ? 1 : 0);
        sl[t].f = T3[op][type];
        sl[t].a = (const char *)in1 + off * esz;
        sl[t].b = (const char *)in2 + off * esz;
        sl[t].o = (char *)out + off * esz;
        sl[t].n = n;
        off += n;
        pthread_create(&th[t], NULL, mt_run, &sl[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return MI355X_SUCCESS;
}

/* ---- reference-signature adapters (op.h:253-266) so tests can install the oracle as the
 *      "base" op component of the mini-OMPI harness.  One adapter per (op,type) slot is
 *      generated at run time through a small thunk table indexed by slot. */
#define NSLOT (MI355X_OP_MAX_ * MI355X_T_MAX)
static int slot_op(int s) { return s / MI355X_T_MAX; }
static int slot_ty(int s) { return s % MI355X_T_MAX; }

#define THUNK(S)                                                                       \
    static void th2_##S(void *in, void *io, int *cnt, void **dt, void *mod)           \
    { (void)dt; (void)mod; T2[slot_op(S)][slot_ty(S)](in, io, (size_t)*cnt); }         \
    static void th3_##S(void *a, void *b, void *o, int *cnt, void **dt, void *mod)    \
    { (void)dt; (void)mod; T3[slot_op(S)][slot_ty(S)](a, b, o, (size_t)*cnt); }
#define THUNK10(B) THUNK(B##0) THUNK(B##1) THUNK(B##2) THUNK(B##3) THUNK(B##4) \
                   THUNK(B##5) THUNK(B##6) THUNK(B##7) THUNK(B##8) THUNK(B##9)
/* 15 ops x 39 types = 585 slots (0..584) */
THUNK10() THUNK10(1) THUNK10(2) THUNK10(3) THUNK10(4) THUNK10(5) THUNK10(6) THUNK10(7)
THUNK10(8) THUNK10(9) THUNK10(10) THUNK10(11) THUNK10(12) THUNK10(13) THUNK10(14)
THUNK10(15) THUNK10(16) THUNK10(17) THUNK10(18) THUNK10(19) THUNK10(20) THUNK10(21)
THUNK10(22) THUNK10(23) THUNK10(24) THUNK10(25) THUNK10(26) THUNK10(27) THUNK10(28)
THUNK10(29) THUNK10(30) THUNK10(31) THUNK10(32) THUNK10(33) THUNK10(34) THUNK10(35)
THUNK10(36) THUNK10(37) THUNK10(38) THUNK10(39) THUNK10(40) THUNK10(41) THUNK10(42)
THUNK10(43) THUNK10(44) THUNK10(45) THUNK10(46) THUNK10(47) THUNK10(48) THUNK10(49)
THUNK10(50) THUNK10(51) THUNK10(52) THUNK10(53) THUNK10(54) THUNK10(55) THUNK10(56)
THUNK10(57) THUNK(580) THUNK(581) THUNK(582) THUNK(583) THUNK(584)

#define REF10(B, K) K##_##B##0, K##_##B##1, K##_##B##2, K##_##B##3, K##_##B##4, \
                    K##_##B##5, K##_##B##6, K##_##B##7, K##_##B##8, K##_##B##9
#define REFALL(K) K##_0, K##_1, K##_2, K##_3, K##_4, K##_5, K##_6, K##_7, K##_8, K##_9,      \
    REF10(1, K), REF10(2, K), REF10(3, K), REF10(4, K), REF10(5, K), REF10(6, K),            \
    REF10(7, K), REF10(8, K), REF10(9, K), REF10(10, K), REF10(11, K), REF10(12, K),         \
    REF10(13, K), REF10(14, K), REF10(15, K), REF10(16, K), REF10(17, K), REF10(18, K),      \
    REF10(19, K), REF10(20, K), REF10(21, K), REF10(22, K), REF10(23, K), REF10(24, K),      \
    REF10(25, K), REF10(26, K), REF10(27, K), REF10(28, K), REF10(29, K), REF10(30, K),      \
    REF10(31, K), REF10(32, K), REF10(33, K), REF10(34, K), REF10(35, K), REF10(36, K),      \
    REF10(37, K), REF10(38, K), REF10(39, K), REF10(40, K), REF10(41, K), REF10(42, K),      \
    REF10(43, K), REF10(44, K), REF10(45, K), REF10(46, K), REF10(47, K), REF10(48, K),      \
    REF10(49, K), REF10(50, K), REF10(51, K), REF10(52, K), REF10(53, K), REF10(54, K),      \
    REF10(55, K), REF10(56, K), REF10(57, K), K##_580, K##_581, K##_582, K##_583, K##_584

static oracle_ompi_fn2_t THK2[] = { REFALL(th2) };
static oracle_ompi_fn3_t THK3[] = { REFALL(th3) };

oracle_ompi_fn2_t oracle_ompi_fn2(int op, int type)
{
    if (!oracle_has_op(op, type)) return NULL;
    return THK2[op * MI355X_T_MAX + type];
}

oracle_ompi_fn3_t oracle_ompi_fn3(int op, int type)
{
    if (!oracle_has_op(op, type)) return NULL;
    return THK3[op * MI355X_T_MAX + type];
}
