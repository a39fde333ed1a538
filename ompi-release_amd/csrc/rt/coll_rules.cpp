// coll_rules.cpp -- coll/tuned's dynamic rules file, read and applied by coll/mi355x.
//
// Format and semantics restated from ompi/mca/coll/tuned/coll_tuned_dynamic_file.c:56-251 (the
// reader), :267-283 (getnext: numbers as fscanf "%li" reads them -- decimal, 0x hex, 0 octal --
// anything else skipped one character at a time, '#' to the end of the line) and
// coll_tuned_dynamic_rules.c:287-393 (the lookups):
//   <number of collectives>
//   for each: <collective id (coll_tuned.h:41-58)> <number of communicator sizes>
//     for each: <communicator size> <number of message sizes>
//       for each: <message size> <algorithm> <fan in/out> <segment size>
// The first message size of every communicator rule must be 0.  For a communicator of size n the
// rule used is the last one, in file order, whose size is <= n (the first one if none is); for a
// message of m bytes, the last message rule with size <= m.  Algorithm 0 = no rule: the forced
// (MCA) algorithm applies, then the fixed decision (coll_tuned_decision_dynamic.c:59-99).
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "rt_internal.hpp"

struct mi355x_rules {
    struct Msg {
        size_t msg_size;
        int alg, faninout, segsize;
    };
    struct Com {
        int comsize;
        std::vector<Msg> msgs;
    };
    std::vector<Com> coll[MI355X_COLL_COUNT];
};

namespace mi355x {
namespace {

struct Reader {
    std::string text;
    size_t pos = 0;
    int line = 1;
    // getnext (coll_tuned_dynamic_file.c:267-283); -1 at the end of the file
    long next()
    {
        for (;;) {
            while (pos < text.size() && isspace((unsigned char)text[pos])) {
                if (text[pos] == '\n') line++;
                pos++;
            }
            if (pos >= text.size()) return -1;
            const char *p = text.c_str() + pos;
            char *end = nullptr;
            const long v = strtol(p, &end, 0);
            if (end != p) {
                pos += (size_t)(end - p);
                return v;
            }
            if (text[pos++] == '#')
                while (pos < text.size() && text[pos] != '\n') pos++;
        }
    }
};

} // namespace
} // namespace mi355x

using namespace mi355x;

extern "C" {

int mi355x_rules_load(const char *path, mi355x_rules_t **out)
{
    if (!path || !out) return set_error(MI355X_ERR_ARG, "NULL argument");
    *out = nullptr;
    FILE *f = fopen(path, "r");
    if (!f) return set_error(MI355X_ERR_ARG, "cannot read rules file [%s]", path);
    Reader rd;
    char buf[4096];
    size_t got;
    while ((got = fread(buf, 1, sizeof(buf), f)) > 0) rd.text.append(buf, got);
    fclose(f);
    auto *r = new mi355x_rules();
    auto fail = [&](const char *what) {
        delete r;
        return set_error(MI355X_ERR_ARG, "rules file %s: %s around line %d", path, what, rd.line);
    };
    const long X = rd.next();
    if (X < 0) return fail("could not read the number of collectives");
    if (X > MI355X_COLL_COUNT) return fail("more collectives than MPI has");
    for (long x = 0; x < X; ++x) {
        const long CI = rd.next();
        if (CI < 0) return fail("could not read a collective id");
        if (CI >= MI355X_COLL_COUNT) return fail("collective id out of range");
        const long NCS = rd.next();
        if (NCS < 0) return fail("could not read the count of communicator sizes");
        std::vector<mi355x_rules::Com> coms((size_t)NCS);
        for (long ncs = 0; ncs < NCS; ++ncs) {
            const long CS = rd.next();
            if (CS < 0) return fail("could not read a communicator size");
            const long NMS = rd.next();
            if (NMS < 0) return fail("could not read the number of message sizes");
            coms[(size_t)ncs].comsize = (int)CS;
            coms[(size_t)ncs].msgs.resize((size_t)NMS);
            for (long nms = 0; nms < NMS; ++nms) {
                const long MS = rd.next();
                if (MS < 0) return fail("could not read a message size");
                const long ALG = rd.next();
                if (ALG < 0) return fail("could not read a target algorithm");
                const long FIO = rd.next();
                if (FIO < 0) return fail("could not read a fan in/out");
                const long SS = rd.next();
                if (SS < 0) return fail("could not read a segment size");
                if (nms == 0 && MS != 0) return fail("the first message size of a communicator rule must be 0");
                coms[(size_t)ncs].msgs[(size_t)nms] = {(size_t)MS, (int)ALG, (int)FIO, (int)SS};
            }
        }
        r->coll[CI] = std::move(coms);
    }
    *out = r;
    return (int)X;
}

int mi355x_rules_destroy(mi355x_rules_t *r)
{
    delete r;
    return MI355X_SUCCESS;
}

int mi355x_rules_decide(const mi355x_rules_t *r, int coll, int comm_size, size_t msg_bytes, int *alg, int *faninout,
                        int *segsize)
{
    if (!alg) return set_error(MI355X_ERR_ARG, "alg is NULL");
    *alg = 0;
    if (!r || coll < 0 || coll >= MI355X_COLL_COUNT) return MI355X_SUCCESS;
    const auto &coms = r->coll[coll];
    if (coms.empty()) return MI355X_SUCCESS;
    // ompi_coll_tuned_get_com_rule_ptr (coll_tuned_dynamic_rules.c:287-325)
    size_t best = 0;
    for (size_t i = 0; i < coms.size(); ++i) {
        if (coms[i].comsize > comm_size) break;
        best = i;
    }
    const auto &msgs = coms[best].msgs;
    if (msgs.empty()) return MI355X_SUCCESS;
    // ompi_coll_tuned_get_target_method_params (:342-393)
    size_t bm = 0;
    for (size_t i = 0; i < msgs.size(); ++i) {
        if (msgs[i].msg_size <= msg_bytes) bm = i;
        else break;
    }
    *alg = msgs[bm].alg;
    if (faninout) *faninout = msgs[bm].faninout;
    if (segsize) *segsize = msgs[bm].segsize;
    return MI355X_SUCCESS;
}

} // extern "C"
