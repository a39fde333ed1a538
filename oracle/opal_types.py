"""opal datatype construction restated -- TEST INFRASTRUCTURE ONLY (imported by tests/ only).

What the reference computes when a derived datatype is built, restated so that the datatype
known-answer tests of test/datatype/opal_datatype_test.c (upper_matrix, mpich_typeub*, test_upper,
the local_copy_with_convertor chunk dances) can be replayed against the GPU convertor:

* bounds, size and flags: opal_datatype_add (opal/datatype/opal_datatype_add.c:103-376) --
  the LB/UB markers (:125-150), OPAL_DATATYPE_LB_UB_CONT (:67-86), the user-marker inheritance
  rule (:186-219), the alignment epsilon when no user UB is set (:221-235), size/true bounds
  (:249-265), the contiguity flags (:352-367); a fresh type (opal_datatype_create.c:35-51) has
  lb = true_lb = LONG_MAX, ub = true_ub = LONG_MIN, align 1; opal_datatype_resize
  (opal_datatype_resize.c:19-30);
* the unoptimized description records (`desc`, 32-byte dt_elem_desc_t, opal_datatype_internal.h:
  148-208) appended by opal_datatype_add (:276-350) and the trailing END_LOOP opal_datatype_commit
  writes (opal_datatype_optimize.c:255-282);
* the constructors as the datatype tests build them (test/datatype/opal_ddt_lib.c:260-475:
  indexed / hindexed / struct / vector / hvector) and opal_datatype_create_contiguous
  (opal_datatype_create_contiguous.c);
* the type map itself (MPI-3.1 §4.1: the basic elements in order), carried independently of the
  description, as the ground truth the pack order follows (opal_datatype_pack.c:250-374).

Predefined types are x86-64 Open MPI's: size = alignment = sizeof (long double 16).
"""
from __future__ import annotations

import struct

LONG_MAX, LONG_MIN = (1 << 63) - 1, -(1 << 63)

# opal_datatype.h:65-82
F_PREDEFINED, F_COMMITTED, F_CONTIGUOUS, F_NO_GAPS = 0x0002, 0x0004, 0x0010, 0x0020
F_USER_LB, F_USER_UB, F_DATA = 0x0040, 0x0080, 0x0100
F_BASIC = F_PREDEFINED | F_CONTIGUOUS | F_NO_GAPS | F_DATA | F_COMMITTED

# opal_datatype_internal.h:107-131
LOOP, END_LOOP, LB, UB = 0, 1, 2, 3
BASIC = {  # name: (id, size = alignment)
    "INT1": (4, 1), "INT2": (5, 2), "INT4": (6, 4), "INT8": (7, 8), "UINT1": (9, 1), "UINT4": (11, 4),
    "FLOAT4": (15, 4), "FLOAT8": (16, 8), "FLOAT16": (18, 16),
}


_PREDEF: dict = {}


def basic_sizes():
    """basic_sizes[type id] for mi355x_ddt_from_opal"""
    s = [0] * 32
    for tid, sz in BASIC.values():
        s[tid] = sz
    return s


class OpalType:
    def __init__(self):  # opal_datatype_construct, opal_datatype_create.c:35-51
        self.size = 0
        self.lb, self.ub = LONG_MAX, LONG_MIN
        self.true_lb, self.true_ub = LONG_MAX, LONG_MIN
        self.align = 1
        self.flags = F_CONTIGUOUS
        self.id = 0
        self.nb_elems = 0
        self.desc: list[tuple] = []   # records; ('E', flags, type, count, extent, disp) / ('L', flags, loops, items, extent) / ('X', flags, items, size, first)
        self.tmap: list[tuple] = []   # (disp, size) per basic element, in type-map order

    # ---- predefined (one object per type, as &opal_datatype_<name> is one address)
    @classmethod
    def basic(cls, name):
        if name not in _PREDEF:
            _PREDEF[name] = cls._basic(name)
        return _PREDEF[name]

    @classmethod
    def _basic(cls, name):
        tid, sz = BASIC[name]
        t = cls()
        t.size, t.lb, t.ub, t.true_lb, t.true_ub, t.align = sz, 0, sz, 0, sz, sz
        t.flags, t.id, t.nb_elems = F_BASIC, tid, 1
        t.desc = [("E", F_BASIC, tid, 1, sz, 0)]  # OPAL_DATATYPE_INIT_DESC_PREDEFINED
        t.tmap = [(0, sz)]
        return t

    @classmethod
    def marker(cls, which):  # opal_datatype_lb / opal_datatype_ub
        t = cls()
        t.id, t.lb, t.ub, t.true_lb, t.true_ub, t.align = which, 0, 0, 0, 0, 0
        t.flags = F_PREDEFINED
        return t

    @property
    def extent(self):
        return self.ub - self.lb

    # ---- opal_datatype_add (opal_datatype_add.c:103-376)
    def add(self, a: "OpalType", count: int, disp: int, extent: int):
        if count == 0:
            return
        if extent == -1:
            extent = a.ub - a.lb
        if a.id == LB:  # :126-137
            self.lb = min(self.lb, disp) if self.flags & F_USER_LB else disp
            self.flags |= F_USER_LB
            if self.ub - self.lb != self.size:
                self.flags &= ~F_NO_GAPS
            return
        if a.id == UB:  # :138-150
            self.ub = max(self.ub, disp) if self.flags & F_USER_UB else disp
            self.flags |= F_USER_UB
            if self.ub - self.lb != self.size:
                self.flags &= ~F_NO_GAPS
            return
        # OPAL_DATATYPE_LB_UB_CONT (:67-86)
        upper, lower = disp + extent * (count - 1), disp
        lb, ub = (lower, upper) if lower < upper else (upper, lower)
        lb += a.lb
        ub += a.ub
        true_lb = lb - (a.lb - a.true_lb)
        true_ub = ub - (a.ub - a.true_ub)
        if true_lb > true_ub:
            true_lb, true_ub = true_ub, true_lb
        # user markers (:186-219)
        if (a.flags ^ self.flags) & F_USER_LB:
            if self.flags & F_USER_LB:
                lb = self.lb
            self.flags |= F_USER_LB
        else:
            lb = min(self.lb, lb)
        if (self.flags ^ a.flags) & F_USER_UB:
            if self.flags & F_USER_UB:
                ub = self.ub
            self.flags |= F_USER_UB
        else:
            ub = max(self.ub, ub)
        self.lb, self.ub = lb, ub
        self.align = max(self.align, a.align)
        if not self.flags & F_USER_UB:  # :230-235
            eps = (self.ub - self.lb) % self.align
            if eps:
                self.ub += self.align - eps
        self.flags |= F_DATA
        if a.size == 0:
            return
        self.size += count * a.size
        old_true_ub = disp if self.nb_elems == 0 else self.true_ub
        self.true_lb = min(true_lb, self.true_lb)
        self.true_ub = max(true_ub, self.true_ub)
        # description records (:276-350)
        if (a.flags & (F_PREDEFINED | F_DATA)) == (F_PREDEFINED | F_DATA):
            if extent != a.size and count > 1:
                lf = a.flags & ~(F_COMMITTED | F_CONTIGUOUS | F_NO_GAPS)
                self.desc += [("L", lf & ~F_DATA, count, 2, extent), ("E", lf | F_CONTIGUOUS, a.id, 1, a.size, disp),
                              ("X", lf & ~F_DATA, 2, a.size, disp)]
            else:
                self.desc.append(("E", a.flags & ~F_COMMITTED, a.id, count, extent, disp))
        else:
            d0 = a.desc[0] if len(a.desc) == 1 else None
            if d0 is not None and d0[0] == "E" and extent == a.ub - a.lb and extent == d0[4]:
                self.desc.append(("E", d0[1], d0[2], d0[3] * count, d0[4], d0[5] + disp))
            else:
                start = len(self.desc)
                if count != 1:
                    self.desc.append(("L", (a.flags & ~F_COMMITTED) & ~F_DATA, count, len(a.desc) + 1, extent))
                for r in a.desc:
                    if r[0] == "E" and r[1] & F_DATA:
                        r = r[:5] + (r[5] + disp,)
                    elif r[0] == "X":
                        r = r[:4] + (r[4] + disp,)
                    self.desc.append(r)
                if count != 1:
                    first = next(r for r in self.desc[start:] if r[0] != "L")
                    self.desc.append(("X", self.desc[start][1], len(a.desc) + 1, a.size, first[5]))
        # contiguity (:352-367)
        lf = self.flags & a.flags
        self.flags &= ~(F_CONTIGUOUS | F_NO_GAPS)
        if (lf & F_CONTIGUOUS) and disp + a.true_lb == old_true_ub and (a.size == extent or count < 2):
            self.flags |= F_CONTIGUOUS
            if self.size == self.ub - self.lb:
                self.flags |= F_NO_GAPS
        self.nb_elems += count * a.nb_elems
        # the type map
        self.tmap += [(disp + i * extent + d, s) for i in range(count) for d, s in a.tmap]

    def resize(self, lb, extent):  # opal_datatype_resize.c:19-30
        self.lb, self.ub = lb, lb + extent
        self.flags &= ~F_NO_GAPS
        if extent == self.size and self.flags & F_CONTIGUOUS:
            self.flags |= F_NO_GAPS
        return self

    def commit(self):  # opal_datatype_optimize.c:255-282 (the optimized copy is not restated)
        self.flags |= F_COMMITTED
        return self

    # ---- outputs
    def desc_bytes(self) -> bytes:
        """the committed `desc` as dt_elem_desc_t records + the trailing END_LOOP commit adds"""
        out = b""
        for r in self.desc:
            if r[0] == "E":
                out += struct.pack("<HHII4xqq", r[1], r[2], r[3], 1, r[4], r[5])
            elif r[0] == "L":
                out += struct.pack("<HHII4xqq", r[1], LOOP, r[2], r[3], -1, r[4])
            else:
                out += struct.pack("<HHII4xQq", r[1], END_LOOP, r[2], 0xFFFFFFFF, r[3], r[4])
        first = next((r[5] for r in self.desc if r[0] == "E"), 0)
        return out + struct.pack("<HHII4xQq", 0, END_LOOP, len(self.desc), 0, self.size, first)

    def runs(self):
        """the type map as merged (disp, len, elem) runs of one instance"""
        out = []
        for d, s in self.tmap:
            if out and out[-1][0] + out[-1][1] == d and out[-1][2] == s:
                out[-1][1] += s
            else:
                out.append([d, s, s])
        return [tuple(r) for r in out]


def contiguous(count, old):  # opal_datatype_create_contiguous.c
    t = OpalType()
    if count:
        t.add(old, count, 0, old.ub - old.lb)
    return t


def vector(count, blen, stride, old):  # opal_ddt_lib.c:414-443
    ext = old.ub - old.lb
    t = OpalType()
    if count == 0:
        return t
    if blen == stride or count <= 1:
        t.add(old, count * blen, 0, ext)
    elif blen == 1:
        t.add(old, count, 0, ext * stride)
    else:
        tmp = OpalType()
        tmp.add(old, blen, 0, ext)
        t.add(tmp, count, 0, ext * stride)
    return t


def hvector(count, blen, stride, old):  # opal_ddt_lib.c:446-475
    ext = old.ub - old.lb
    t = OpalType()
    if count == 0:
        return t
    if ext * blen == stride or count <= 1:
        t.add(old, count * blen, 0, ext)
    elif blen == 1:
        t.add(old, count, 0, stride)
    else:
        tmp = OpalType()
        tmp.add(old, blen, 0, ext)
        t.add(tmp, count, 0, stride)
    return t


def indexed(blens, disps, old):  # opal_ddt_lib.c:260-300 (adjacent blocks merge)
    ext = old.ub - old.lb
    t = OpalType()
    if not blens:
        return t
    disp, dlen = disps[0], blens[0]
    endat = disp + dlen
    if len(blens) == 1:
        t.add(old, dlen, disp * ext, ext)
        return t
    for b, d in zip(blens[1:], disps[1:]):
        if endat == d:
            dlen += b
            endat += b
        else:
            t.add(old, dlen, disp * ext, ext)
            disp, dlen, endat = d, b, d + b
    t.add(old, dlen, disp * ext, ext)
    return t


def hindexed(blens, disps, old):  # opal_ddt_lib.c:302-342
    ext = old.ub - old.lb
    t = OpalType()
    if not blens:
        return t
    disp, dlen = disps[0], blens[0]
    endat = disp + dlen * ext
    if len(blens) == 1:
        t.add(old, dlen, disp, ext)
        return t
    for b, d in zip(blens[1:], disps[1:]):
        if endat == d:
            dlen += b
            endat += b * ext
        else:
            t.add(old, dlen, disp, ext)
            disp, dlen, endat = d, b, d + b * ext
    t.add(old, dlen, disp, ext)
    return t


def struct_(blens, disps, types):  # opal_ddt_lib.c:345-411 (same type at the running end merges)
    t = OpalType()
    if not blens:
        return t
    last, lblk, ldisp = types[0], blens[0], disps[0]
    lext = last.ub - last.lb
    endto = ldisp + lext * lblk
    for b, d, ty in zip(blens[1:], disps[1:], types[1:]):
        if ty is last and d == endto:
            lblk += b
            endto = ldisp + lblk * lext
        else:
            t.add(last, lblk, ldisp, lext)
            last, lblk, ldisp = ty, b, d
            lext = last.ub - last.lb
            endto = ldisp + lext * lblk
    t.add(last, lblk, ldisp, lext)
    return t


# ---- the types of test/datatype/opal_ddt_lib.c / opal_datatype_test.c
def upper_matrix(n):  # opal_ddt_lib.c:514-544
    return indexed([n - i for i in range(n)], [i * n + i for i in range(n)], OpalType.basic("FLOAT8")).commit()


def strange_dt():  # opal_ddt_lib.c:203-234 (USE_RESIZED; sizeof(sdata_intern) = 12)
    p = OpalType()
    p.add(OpalType.basic("FLOAT8"), 1, 0, -1)
    p.add(OpalType.basic("INT1"), 1, 8, -1)
    p.resize(0, 12)
    return contiguous(10, p).commit()


def struct_char_double():  # opal_ddt_lib.c:168-186 ({char c; double d;}: d at 8)
    return struct_([1, 1], [0, 8], [OpalType.basic("INT1"), OpalType.basic("FLOAT8")]).commit()


def twice_two_doubles():  # opal_ddt_lib.c:58-68
    return vector(2, 2, 5, OpalType.basic("FLOAT8")).commit()


BLACS_LEN = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
BLACS_IDX = [x // 4 for x in (1144, 1232, 1320, 1408, 1496, 1584, 1676, 1768, 1860, 1952, 2044, 2136, 2228,
                              2320, 2412, 2504, 2596, 2688)]


def blacs():  # opal_ddt_lib.c:95-109
    return indexed(BLACS_LEN, BLACS_IDX, OpalType.basic("INT4")).commit()


def blacs1():  # :111-121
    return vector(7, 1, 3, OpalType.basic("INT4")).commit()


def blacs2():  # :123-133
    return vector(7, 1, 2, OpalType.basic("INT4")).commit()


def test_struct():  # opal_ddt_lib.c:136-161
    p = OpalType()
    p.add(OpalType.basic("FLOAT8"), 1, 0, -1)
    p.add(OpalType.basic("INT1"), 1, 8, -1)
    return struct_([2, 1, 3], [0, 16, 26], [OpalType.basic("FLOAT4"), p, OpalType.basic("INT1")]).commit()


def contiguous_alignment():  # test_contiguous, opal_ddt_lib.c:590-615
    p = OpalType()
    p.add(OpalType.basic("FLOAT8"), 1, 0, -1)
    p.add(OpalType.basic("INT1"), 1, 8, -1)
    return contiguous(2, contiguous(4, p)).commit()


def matrix_borders(size, width):  # opal_ddt_lib.c:571-587 (disp[1] counted in doubles by indexed)
    line = indexed([width, width], [0, (size - width) * 8], OpalType.basic("FLOAT8"))
    return contiguous(size, line).commit()


def typeub():  # mpich_typeub, opal_ddt_lib.c:619-679 -> extents of type1, type2, type3
    t1 = vector(2, 1, 4, OpalType.basic("INT4")).commit()
    t2 = struct_([1, 1], [0, 16], [t1, OpalType.marker(UB)]).commit()
    t3 = struct_([1, 1], [0, 4], [t2, OpalType.marker(UB)]).commit()
    return t1, t2, t3


def typeub_dt1():  # the {LB -3, int 0, UB 6} type of mpich_typeub2/3 (:688-699, :768-780)
    return struct_([1, 1, 1], [-3, 0, 6], [OpalType.marker(LB), OpalType.basic("INT4"), OpalType.marker(UB)]).commit()


def typeub2():  # :681-758 -> dt1, contiguous(2, dt1), struct{dt1 at 0, dt1 at ex1}
    dt1 = typeub_dt1()
    dt2 = contiguous(2, dt1).commit()
    dt3 = struct_([1, 1], [0, dt1.extent], [dt1, dt1]).commit()
    return dt1, dt2, dt3


def typeub3():  # :760-850 -> hindexed, indexed, hvector, vector of dt1
    dt1 = typeub_dt1()
    return (hindexed([1, 1], [-4, 7], dt1).commit(), indexed([1, 1], [-4, 7], dt1).commit(),
            hvector(2, 1, 14, dt1).commit(), vector(2, 1, 14, dt1).commit())


def walk_desc(t: OpalType, count: int = 1):
    """the basic elements in the order the convertor visits them walking `desc` (the stack walk of
    opal_generic_simple_pack, opal_datatype_pack.c:250-374: ELEM = `count` elements `extent`
    apart, LOOP = its body `loops` times `extent` apart, instance k at k * (ub - lb))"""
    sizes = basic_sizes()
    recs = t.desc
    out = []

    def body(i, end, base):
        while i < end:
            r = recs[i]
            if r[0] == "L":
                stop = i + r[3]  # index of the matching END_LOOP
                for k in range(r[2]):
                    body(i + 1, stop, base + k * r[4])
                i = stop + 1
            elif r[0] == "E":
                out.extend((base + r[5] + c * r[4], sizes[r[2]]) for c in range(r[3]))
                i += 1
            else:
                i += 1

    for k in range(count):
        body(0, len(recs), k * t.extent)
    return out


def convertor_raw(t: OpalType, count: int = 1, iov_num: int = 5):
    """opal_convertor_raw (opal/datatype/opal_convertor_raw.c:37-180) over the restated records:
    the iovecs the reference hands back, one list per call of at most `iov_num` entries (the
    function stops when the iovec array is full and resumes there on the next call; the last call
    returns 1).  Emission rules: a data ELEM whose extent equals its basic size is one iovec of
    count * size (:87-101), any other ELEM one iovec per element (:102-114); a LOOP flagged
    CONTIGUOUS one iovec of the END_LOOP's size per iteration at first_elem_disp (:145-158); any
    other LOOP is walked into; instance k at k * (ub - lb) (:131).  (The reference walks opt_desc
    for a homogeneous convertor; the optimized records are not restated -- the same bytes in the
    same order, possibly cut into different iovecs.)"""
    sizes = basic_sizes()
    recs = t.desc
    flat = []

    def body(i, end, base):
        while i < end:
            r = recs[i]
            if r[0] == "L":
                stop = i + r[3]  # the matching END_LOOP
                if r[1] & F_CONTIGUOUS:
                    x = recs[stop]
                    flat.extend((base + x[4] + k * r[4], x[3]) for k in range(r[2]))
                else:
                    for k in range(r[2]):
                        body(i + 1, stop, base + k * r[4])
                i = stop + 1
            elif r[0] == "E":
                if r[1] & F_DATA:
                    sz = sizes[r[2]]
                    if sz == r[4]:
                        flat.append((base + r[5], sz * r[3]))
                    else:
                        flat.extend((base + r[5] + c * r[4], sz) for c in range(r[3]))
                i += 1
            else:
                i += 1

    for k in range(count):
        body(0, len(recs), k * t.extent)
    flat = [p for p in flat if p[1]]
    return [flat[i:i + iov_num] for i in range(0, len(flat), iov_num)] or [[]]


def merge_pieces(pieces):
    """adjacent (offset, length) pieces merged: the byte sequence they describe"""
    out = []
    for d, n in pieces:
        if out and out[-1][0] + out[-1][1] == d:
            out[-1][1] += n
        else:
            out.append([d, n])
    return [tuple(p) for p in out]


def ddt_test_zero_count_types():
    """test/datatype/ddt_test.c:401-411: three types grown from contiguous(0, MPI_DATATYPE_NULL)
    by ompi_datatype_add -- pdt3 = 10 int + 5 float at 40; pdt2 = float + 3 x pdt3 at 4; pdt1 =
    5 long long + 2 long double at 40 (returns pdt1, pdt2, pdt3)"""
    i4, f4, i8, f16 = (OpalType.basic(n) for n in ("INT4", "FLOAT4", "INT8", "FLOAT16"))
    p3 = contiguous(0, i4)
    p3.add(i4, 10, 0, -1)
    p3.add(f4, 5, 10 * 4, -1)
    p2 = contiguous(0, i4)
    p2.add(f4, 1, 0, -1)
    p2.add(p3, 3, 4, -1)
    p1 = contiguous(0, i4)
    p1.add(i8, 5, 0, -1)
    p1.add(f16, 2, 8 * 5, -1)
    return p1.commit(), p2.commit(), p3.commit()


def inversed_vector(length):  # create_inversed_vector, test/datatype/ddt_lib.c:59-67 (vector(length, 1, 2, int))
    return vector(length, 1, 2, OpalType.basic("INT4")).commit()
