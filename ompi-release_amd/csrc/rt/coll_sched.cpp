// coll_sched.cpp -- symbolic re-execution of the coll/tuned schedules (see coll_sched.hpp).
#include "coll_sched.hpp"

#include <algorithm>
#include <functional>

namespace mi355x {

// ----------------------------------------------------------------- expression -> program
bool compile_expr(const ExprPool &p, int root, int n, Program *out)
{
    *out = Program();
    out->nr = n;
    // 1) chain (left-deep) form -> k_fold
    {
        std::vector<int> ranks;   // collected from the root down
        std::vector<int> roles;
        int cur = root;
        bool ok = true;
        while (p.e[cur].rank < 0) {
            const Expr &x = p.e[cur];
            if (p.e[x.out].rank >= 0) {        // op2(out = x_leaf, in = acc)
                ranks.push_back(p.e[x.out].rank);
                roles.push_back(0);
                cur = x.in;
            } else if (p.e[x.in].rank >= 0) {  // op2(out = acc, in = x_leaf)
                ranks.push_back(p.e[x.in].rank);
                roles.push_back(1);
                cur = x.out;
            } else {
                ok = false;
                break;
            }
        }
        if (ok) {
            ranks.push_back(p.e[cur].rank);
            roles.push_back(0);
            std::reverse(ranks.begin(), ranks.end());
            std::reverse(roles.begin(), roles.end());
            if ((int)ranks.size() <= kMaxRanks) {
                out->is_fold = true;
                out->order = ranks;
                out->role_mask = 0;
                for (size_t j = 1; j < roles.size(); ++j)
                    if (roles[j]) out->role_mask |= (1ull << j);
                return true;
            }
        }
    }
    // 2) general tree -> register program; every leaf is used exactly once, so the register of
    //    a node's `out` operand can hold its result.
    if (n > kTreeMax) return false;
    std::function<int(int)> emit = [&](int id) -> int {
        const Expr &x = p.e[id];
        if (x.rank >= 0) return x.rank;
        const int ro = emit(x.out);
        const int ri = emit(x.in);
        out->steps.push_back({(int8_t)ro, (int8_t)ro, (int8_t)ri});
        return ro;
    };
    out->result = emit(root);
    return (int)out->steps.size() <= kTreeSteps;
}

// ----------------------------------------------------------------- allreduce
static int largest_pow2_le(int n)
{
    int p = 1;
    while ((p << 1) <= n) p <<= 1;
    return p;
}

int expr_allreduce_recursive_doubling(ExprPool &p, int n)
{
    // coll_tuned_allreduce.c:143-294, with buffers as expression ids
    std::vector<int> tsend(n), newrank(n);
    for (int r = 0; r < n; ++r) tsend[r] = p.leaf(r);
    if (n == 1) return tsend[0];
    const int adjsize = largest_pow2_le(n);   // opal_next_poweroftwo(size) >> 1
    const int extra = n - adjsize;
    for (int r = 0; r < n; ++r) {
        if (r < 2 * extra) {
            if (r % 2 == 0) {
                newrank[r] = -1;
            } else {
                // tmpsend = tmprecv (op) tmpsend: target tmpsend (:214-217)
                tsend[r] = p.op(tsend[r], tsend[r - 1]);
                newrank[r] = r >> 1;
            }
        } else {
            newrank[r] = r - extra;
        }
    }
    for (int dist = 1; dist < adjsize; dist <<= 1) {
        std::vector<int> next = tsend;
        for (int r = 0; r < n; ++r) {
            if (newrank[r] < 0) continue;
            const int nr = newrank[r] ^ dist;
            const int remote = (nr < extra) ? nr * 2 + 1 : nr + extra;
            const int mine = tsend[r], theirs = tsend[remote];
            // rank < remote: tmprecv = tmpsend (op) tmprecv -> out = received (:248-254)
            // else          : tmpsend = tmprecv (op) tmpsend -> out = mine     (:255-257)
            next[r] = (r < remote) ? p.op(theirs, mine) : p.op(mine, theirs);
        }
        tsend = next;
    }
    // even ranks < 2*extra receive the result of rank+1 (:265-278)
    return tsend[(n > 1 && 0 < 2 * extra) ? 1 : 0];
}

Program ring_block_program(int n, int b)
{
    // block b leaves rank b first; every later rank computes rbuf[b] = inbuf (op) rbuf[b], i.e.
    // op2(out = its local value, in = received partial) (coll_tuned_allreduce.c:480-496, :506-512)
    Program pr;
    pr.is_fold = true;
    pr.nr = n;
    for (int j = 0; j < n; ++j) pr.order.push_back((b + j) % n);
    pr.role_mask = 0;
    return pr;
}

Program reduce_scatter_ring_block_program(int n, int b)
{
    // coll_tuned_reduce_scatter.c:560-615: rank r first sends block r-1 (its own data), then at
    // step k reduces block r-k as accum = inbuf (op) accum (out = local), and finally block r.
    // Block b therefore starts at rank b+1 and ends at rank b.
    Program pr;
    pr.is_fold = true;
    pr.nr = n;
    for (int j = 1; j <= n; ++j) pr.order.push_back((b + j) % n);
    pr.role_mask = 0;
    return pr;
}

std::vector<int> expr_reduce_scatter_rechalving(ExprPool &p, int n)
{
    // ompi_coll_tuned_reduce_scatter_intra_basic_recursivehalving (coll_tuned_reduce_scatter.c:
    // 141-400), per original rank-block; every reduction is
    // ompi_op_reduce(op, recv_buf, result_buf): out = own result, in = received.
    std::vector<std::vector<int>> res(n, std::vector<int>(n));
    for (int r = 0; r < n; ++r)
        for (int b = 0; b < n; ++b) res[r][b] = p.leaf(r);
    const int tmp_size = largest_pow2_le(n), remain = n - tmp_size;
    std::vector<int> tmp_rank(n);
    for (int r = 0; r < n; ++r) {
        if (r < 2 * remain) {
            if ((r & 1) == 0) {
                tmp_rank[r] = -1;
            } else {
                for (int b = 0; b < n; ++b) res[r][b] = p.op(res[r][b], res[r - 1][b]);
                tmp_rank[r] = r / 2;
            }
        } else {
            tmp_rank[r] = r - remain;
        }
    }
    // tmp block i covers original blocks {2i, 2i+1} for i < remain, else {i + remain}
    auto tmp_blocks = [&](int lo, int hi, std::vector<int> &out) {
        for (int i = lo; i < hi; ++i) {
            if (i < remain) {
                out.push_back(2 * i);
                out.push_back(2 * i + 1);
            } else {
                out.push_back(i + remain);
            }
        }
    };
    std::vector<int> send_index(n, 0), recv_index(n, 0), last_index(n, tmp_size);
    for (int mask = tmp_size >> 1; mask > 0; mask >>= 1) {
        std::vector<std::vector<int>> next = res;
        for (int r = 0; r < n; ++r) {
            const int tr = tmp_rank[r];
            if (tr < 0) continue;
            const int tp = tr ^ mask;
            const int peer = (tp < remain) ? tp * 2 + 1 : tp + remain;
            int rlo, rhi;
            if (tr < tp) {
                send_index[r] = recv_index[r] + mask;
                rlo = recv_index[r];
                rhi = send_index[r];
            } else {
                recv_index[r] = send_index[r] + mask;
                rlo = recv_index[r];
                rhi = last_index[r];
            }
            std::vector<int> blks;
            tmp_blocks(rlo, rhi, blks);
            for (int b : blks) next[r][b] = p.op(res[r][b], res[peer][b]);
            send_index[r] = recv_index[r];
            last_index[r] = recv_index[r] + mask;
        }
        res = next;
    }
    // owner of block b: rank b itself, or (even b < 2*remain) the odd neighbour b+1 (:381-397)
    std::vector<int> out(n);
    for (int b = 0; b < n; ++b) out[b] = (b < 2 * remain && (b & 1) == 0) ? res[b + 1][b] : res[b][b];
    return out;
}

// ----------------------------------------------------------------- reduce trees
static int pown(int f, int k)
{
    int v = 1;
    for (int i = 0; i < k; ++i) v *= f;
    return v;
}
static int calc_level(int f, int r)
{
    int level = 0, num = 0;
    for (; num <= r; ++level) num += pown(f, level);
    return level - 1;
}

// ompi_coll_tuned_topo_build_chain(fanout, comm, root) (coll_tuned_topo.c:457-603): children of
// `rank`; the non-root ranks form `fanout` chains hanging off the root
static void chain_children(int fanout, int n, int root, int sr, std::vector<int> &ch)
{
    if (fanout < 1) fanout = 1;
    if (fanout > 32) fanout = 32;  // MAXTREEFANOUT
    if (n - 1 < fanout) fanout = n - 1;
    if (fanout == 1) {
        if (sr + 1 < n) ch.push_back((sr + 1 + root) % n);
        return;
    }
    if (n == 1) return;
    int maxchainlen = (n - 1) / fanout, mark;
    if ((n - 1) % fanout != 0) {
        maxchainlen++;
        mark = (n - 1) % fanout;
    } else {
        mark = fanout + 1;
    }
    if (sr == 0) {  // the root: the heads of the chains (:584-594)
        int next = (root + 1) % n;
        ch.push_back(next);
        for (int i = 1; i < fanout; ++i) {
            next += maxchainlen;
            if (i > mark) next--;
            next %= n;
            ch.push_back(next);
        }
        return;
    }
    int head, len;  // (:550-579)
    if (sr - 1 < mark * maxchainlen) {
        const int column = (sr - 1) / maxchainlen;
        head = 1 + column * maxchainlen;
        len = maxchainlen;
    } else {
        const int column = mark + (sr - 1 - mark * maxchainlen) / (maxchainlen - 1);
        head = mark * maxchainlen + 1 + (column - mark) * (maxchainlen - 1);
        len = maxchainlen - 1;
    }
    if (sr != head + len - 1 && sr + 1 < n) ch.push_back((sr + 1 + root) % n);
}

static std::vector<int> children(int alg, int n, int root, int rank, int chain_fanout)
{
    std::vector<int> ch;
    int sr = rank - root;
    if (sr < 0) sr += n;
    switch (alg) {
    case RED_LINEAR:
    case RED_PIPELINE:
        // fanout-1 chain (coll_tuned_topo.c:515-527); linear has the order of the chain rooted
        // at rank 0 whatever the root (coll_tuned_reduce.c:673-703)
        chain_children(1, n, root, sr, ch);
        break;
    case RED_CHAIN:
        chain_children(chain_fanout, n, root, sr, ch);
        break;
    case RED_BINARY: {
        // ompi_coll_tuned_topo_build_tree(2, ...) (coll_tuned_topo.c:76-189)
        if (n < 2) break;
        const int level = calc_level(2, sr), delta = pown(2, level);
        for (int i = 0; i < 2; ++i) {
            const int sc = sr + delta * (i + 1);
            if (sc < n) ch.push_back((sc + root) % n);
            else break;
        }
        break;
    }
    case RED_BINOMIAL: {
        // ompi_coll_tuned_topo_build_bmtree (coll_tuned_topo.c:324-398)
        int mask = 1;
        while (mask <= sr) mask <<= 1;  // opal_next_poweroftwo(index)
        while (mask < n) {
            int remote = sr ^ mask;
            if (remote >= n) break;
            remote += root;
            if (remote >= n) remote -= n;
            ch.push_back(remote);
            mask <<= 1;
        }
        break;
    }
    }
    return ch;
}

int expr_reduce(ExprPool &p, int alg, int n, int root, int chain_fanout)
{
    // ompi_coll_tuned_reduce_generic (coll_tuned_reduce.c:66-361), commutative op, not in place:
    //   one child : acc = child (op) own          (child received into accumbuf, :150-160, :211-221)
    //   k children: acc = ((c0 (op) own) (op) c1) ... (op) c(k-1)                      (:189-222)
    const int top = (alg == RED_LINEAR) ? 0 : root;
    std::function<int(int)> eval = [&](int r) -> int {
        const std::vector<int> ch = children(alg, n, alg == RED_LINEAR ? 0 : root, r, chain_fanout);
        if (ch.empty()) return p.leaf(r);
        int acc = p.op(eval(ch[0]), p.leaf(r));
        for (size_t i = 1; i < ch.size(); ++i) acc = p.op(acc, eval(ch[i]));
        return acc;
    };
    return eval(top);
}

// ----------------------------------------------------------------- decisions
int allreduce_decision(int n, size_t count, size_t dsize)
{
    const size_t bytes = dsize * count;
    if (bytes < 10000) return AR_RECDBL;
    if (count > (size_t)n) {
        const size_t seg = 1u << 20;
        return ((size_t)n * seg >= bytes) ? AR_RING : AR_RING_SEGMENTED;
    }
    return AR_NONOVERLAPPING;
}

int reduce_decision(int n, size_t count, size_t dsize)
{
    const double a1 = 0.6016 / 1024.0, b1 = 1.3496, a2 = 0.0410 / 1024.0, b2 = 9.7128;
    const double a3 = 0.0422 / 1024.0, b3 = 1.1614, a4 = 0.0033 / 1024.0, b4 = 1.6761;
    const size_t msg = dsize * count;
    (void)a4; (void)b4;
    if (n < 8 && msg < 512) return RED_LINEAR;
    if ((n < 8 && msg < 20480) || msg < 2048 || count <= 1) return RED_BINOMIAL;
    if (n > a1 * (double)msg + b1) return RED_BINOMIAL;
    if (n > a2 * (double)msg + b2) return RED_PIPELINE;
    if (n > a3 * (double)msg + b3) return RED_BINARY;
    return RED_PIPELINE;  // Pipeline_32K or Pipeline_64K: same order
}

int reduce_scatter_decision(int n, size_t total_count, size_t dsize)
{
    const double a = 0.0012, b = 8.0;
    const size_t small = 12 * 1024, large = 256 * 1024;
    const size_t total = total_count * dsize;
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    if (total <= small || (total <= large && pow2 == n) || (n >= a * (double)total + b)) return RS_RECHALVING;
    return RS_RING;
}

size_t computed_segcount(size_t segsize, size_t typelng, size_t count)
{
    if (segsize >= typelng && segsize < typelng * count) {
        size_t sc = segsize / typelng;
        if (segsize - sc * typelng > (typelng >> 1)) sc++;
        return sc;
    }
    return count;
}

void ring_block(size_t count, int n, int b, size_t *off, size_t *len)
{
    size_t early = count / (size_t)n, late = early, split = count % (size_t)n;
    if (split) early += 1;
    *off = ((size_t)b < split) ? (size_t)b * early : (size_t)b * late + split;
    *len = ((size_t)b < split) ? early : late;
}

} // namespace mi355x
