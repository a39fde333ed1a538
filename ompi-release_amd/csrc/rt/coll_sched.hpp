// coll_sched.hpp -- schedule compiler of coll/mi355x.
//
// The reference's per-element result is fixed by the order in which its point-to-point
// schedule applies ompi_op_reduce(op, source, target) (target = target (op) source,
// ompi/op/op.h:540-574).  This compiler re-runs each schedule of coll/tuned SYMBOLICALLY --
// buffers hold expression ids instead of data -- and turns the resulting expression tree into a
// device program: a left fold (k_fold) when the tree is a chain, a register program (k_tree)
// otherwise.  The device then evaluates that exact tree per element, reading every rank's input
// over xGMI, so float results match the reference's schedule bit for bit without moving data
// the way the reference does.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "coll_internal.hpp"

namespace mi355x {

struct Expr {
    int rank;       // >= 0: leaf (that rank's input); -1: op node
    int out, in;    // op node: op2(out = pool[out], in = pool[in])
};

struct ExprPool {
    std::vector<Expr> e;
    int leaf(int r) { e.push_back({r, -1, -1}); return (int)e.size() - 1; }
    int op(int out, int in) { e.push_back({-1, out, in}); return (int)e.size() - 1; }
};

// A compiled per-element program.
struct Program {
    bool is_fold = false;
    // fold form
    std::vector<int> order;     // ranks, acc starts at order[0]
    uint64_t role_mask = 0;     // bit j: acc is the `out` operand at step j
    // tree form
    std::vector<TreeStep> steps;
    int result = 0;
    int nr = 0;                 // ranks referenced (inputs 0..nr-1)
};

// compile an expression tree rooted at `root` over ranks [0, n)
bool compile_expr(const ExprPool &p, int root, int n, Program *out);

// ---- reference schedules, restated symbolically ----------------------------------------------
// MPI_Allreduce, recursive doubling (coll_tuned_allreduce.c:143-294): expression of the result
// (identical on every rank).
int expr_allreduce_recursive_doubling(ExprPool &p, int n);
// Ring / segmented ring (coll_tuned_allreduce.c:360-554, :635-873): element of block b ends as
// ((x_b (op) x_{b+1}) ...) with each later rank's LOCAL value as `out` and the received partial
// as `in` (:480-496).
Program ring_block_program(int n, int b);
// MPI_Reduce trees (coll_tuned_reduce.c:66-361, :618-721; topologies coll_tuned_topo.c).
// The chain (alg 2) hangs `chain_fanout` chains off the root (coll_tuned_topo.c:457-603); the
// reference's value is the MCA parameter coll_tuned_reduce_algorithm_chain_fanout (default 4,
// coll_tuned_component.c:51) or the fan-in/out of a dynamic rule.
enum ReduceAlg { RED_LINEAR = 1, RED_CHAIN = 2, RED_PIPELINE = 3, RED_BINARY = 4, RED_BINOMIAL = 5 };
constexpr int kDefaultChainFanout = 4;
int expr_reduce(ExprPool &p, int alg, int n, int root, int chain_fanout = kDefaultChainFanout);
// MPI_Reduce_scatter recursive halving (coll_tuned_reduce_scatter.c:141-400): expression of
// every rank block b (independent of rcounts).
std::vector<int> expr_reduce_scatter_rechalving(ExprPool &p, int n);
// MPI_Reduce_scatter ring (coll_tuned_reduce_scatter.c:466-636): program of block b.
Program reduce_scatter_ring_block_program(int n, int b);

// ---- decisions (coll_tuned_decision_fixed.c) --------------------------------------------------
enum AllreduceAlg { AR_DECISION = 0, AR_LINEAR = 1, AR_NONOVERLAPPING = 2, AR_RECDBL = 3, AR_RING = 4,
                    AR_RING_SEGMENTED = 5 };
int allreduce_decision(int n, size_t count, size_t dsize);            // :42-85
int reduce_decision(int n, size_t count, size_t dsize);               // :343-446 (commutative)
// reduce_scatter algorithm ids of coll/tuned (coll_tuned_reduce_scatter.c:46-52)
enum ReduceScatterAlg { RS_NONOVERLAPPING = 1, RS_RECHALVING = 2, RS_RING = 3 };
int reduce_scatter_decision(int n, size_t total_count, size_t dsize); // :456-502; RS_RECHALVING or RS_RING

// COLL_TUNED_COMPUTED_SEGCOUNT (coll_tuned.h:525-533)
size_t computed_segcount(size_t segsize, size_t typelng, size_t count);
// COLL_TUNED_COMPUTE_BLOCKCOUNT (coll_tuned.h:546-552) block offset/length
void ring_block(size_t count, int n, int b, size_t *off, size_t *len);

} // namespace mi355x
