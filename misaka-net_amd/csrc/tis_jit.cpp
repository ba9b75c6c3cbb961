// tis_jit.cpp -- code generator of tier 3 (see tis_jit.h).  Host C++ only:
// it produces source text; mk_exec.hip compiles it with hiprtc and the check
// library (sched_check.cpp) exposes the lane function to the CPU tests, which
// compile it with g++ and compare it with the oracle.
//
// The input is the device form of the schedule (assemble_device with 8-byte
// register stride, so register r has operand r*8) -- the same stream the
// tier-2 kernel interprets and the host model in sched_check.cpp executes --
// and each micro-op is restated exactly as those two execute it.
//
// Two shapes of generated code (tis_jit.h):
//   stream  -- the reachable superblock graph is acyclic: every lane runs a
//              bounded straight-line path, so the kernel streams tiles of 4
//              lanes per thread with vector I/O (HBM-bound networks);
//   machine -- the graph has cycles (loops whose trip counts follow the
//              data): each thread holds one lane as a small state machine
//              (superblock id + registers), a wave-uniform dispatcher runs
//              one superblock at a time for the lanes sitting on it (rounds),
//              or every superblock in turn in forward order (sweeps, machines
//              of kSweepMinVariants or more), and a lane that ends takes its
//              next input while the others go on.
#include "tis_jit.h"

#include <algorithm>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/mk.h"

namespace mk {

namespace {

#define MK_DEVICE_SRC(...) #__VA_ARGS__
const char *const kDeviceCommon =
#include "mk_device_common.inc"
    ;
#undef MK_DEVICE_SRC

struct Emitter {
    std::string s;
    void line(const char *fmt, ...) __attribute__((format(printf, 2, 3)))
    {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        s += buf;
        s += '\n';
    }
};

std::string u64lit(int64_t v)
{
    char b[32];
    snprintf(b, sizeof b, "0x%016" PRIx64 "ull", (uint64_t)v);
    return b;
}

// A stretch of a superblock that repeats: `reps` copies of `period`
// micro-ops that are identical except for stack-slot numbers (ST/LD/STI)
// and round-end step counts (ROUND_END), which advance by a fixed amount
// per copy.  The schedule compiler unrolls every loop whose control is
// constant (a PUSH loop of 64: 64 copies of its body, one slot apart); the
// generator rolls such stretches back into `for` loops, which keeps the
// source small enough for hiprtc (a straight-line 23K-op lane takes minutes
// to compile) at the cost of an index computation per slot access.
struct Run {
    size_t start = 0, period = 0, reps = 0;
    std::vector<int64_t> delta; // per op of the period: slot or step advance per copy
    std::vector<Run> inner;     // runs inside the first copy (nested loops)
};

// The reachable part of a schedule's device form.
struct Graph {
    std::vector<DOp> D;
    std::vector<uint32_t> entry;
    std::vector<char> seen;      // variant reachable from variant 0
    std::vector<char> used_reg;  // register read or written by reachable code
    std::vector<char> narrow;    // register whose high 32 bits nothing reads (narrow_regs): uint32_t
    size_t nreach = 0, ndops = 0; // ndops: micro-ops emitted (rolled runs count once)
    bool cyclic = false;
    std::vector<std::vector<uint32_t>> succ; // per reachable variant, its exits' targets
    std::vector<std::vector<Run>> runs; // per variant, ascending start
    const JitLimits *lim = nullptr;
};

bool slot_op(const DOp &I) { return I.op == U_ST || I.op == U_LD || I.op == U_STI; }

// The advancing field of an op: slot for ST/LD (imm) and STI (d), step count
// for ROUND_END (inc); -1 for ops without one.
int64_t advancing(const DOp &I)
{
    if (I.op == U_ST || I.op == U_LD) return (int64_t)(uint32_t)I.imm;
    if (I.op == U_STI) return I.d;
    if (I.op == U_ROUND_END) return I.inc;
    return -1;
}

// Equal apart from the advancing field.
bool same_shape(const DOp &x, const DOp &y)
{
    if (x.op != y.op || x.fl != y.fl || x.a != y.a || x.b != y.b) return false;
    switch (x.op) {
    case U_ST: case U_LD: return x.d == y.d;
    case U_STI: return x.imm == y.imm;
    case U_ROUND_END: return x.d == y.d && x.imm == y.imm;
    default: return x.d == y.d && x.imm == y.imm && x.inc == y.inc;
    }
}

constexpr size_t kRunMaxPeriod = 512, kRunMinReps = 3, kRunMinOps = 24;

// Greedy roll-up of the body [lo, hi) of one variant (data ops and ROUND_END),
// nested: each run's first copy is rolled again.  `outer` are the enclosing
// runs: an op inside a run must advance by the same amount per enclosing
// copy in every copy of the run, so that one affine expression covers it.
std::vector<Run> find_runs(const std::vector<DOp> &D, size_t lo, size_t hi, std::vector<const Run *> &outer)
{
    auto same_outer = [&](size_t a, size_t b) {
        for (const Run *o : outer)
            if (o->delta[a - o->start] != o->delta[b - o->start]) return false;
        return true;
    };
    std::vector<Run> out;
    size_t i = lo;
    while (i < hi) {
        Run best;
        const size_t pmax = std::min(kRunMaxPeriod, (hi - i) / kRunMinReps);
        for (size_t P = 1; P <= pmax; ++P) {
            if (!same_shape(D[i], D[i + P])) continue;
            // deltas from the first two copies
            std::vector<int64_t> dl(P);
            bool ok = true;
            for (size_t k = 0; k < P && ok; ++k) {
                const DOp &x = D[i + k], &y = D[i + P + k];
                ok = same_shape(x, y) && same_outer(i + k, i + P + k);
                const int64_t ax = advancing(x), ay = advancing(y);
                dl[k] = ax >= 0 ? ay - ax : 0;
            }
            if (!ok) continue;
            size_t r = 2;
            for (;; ++r) {
                if (i + (r + 1) * P > hi) break;
                bool m = true;
                for (size_t k = 0; k < P && m; ++k) {
                    const DOp &x = D[i + k], &y = D[i + r * P + k];
                    m = same_shape(x, y) && same_outer(i + k, i + r * P + k) &&
                        (advancing(x) < 0 || advancing(y) == advancing(x) + (int64_t)r * dl[k]);
                }
                if (!m) break;
            }
            if (r >= kRunMinReps && r * P >= kRunMinOps && r * P > best.reps * best.period) {
                best.start = i;
                best.period = P;
                best.reps = r;
                best.delta = dl;
            }
        }
        if (best.reps) {
            outer.push_back(&best);
            best.inner = find_runs(D, best.start, best.start + best.period, outer);
            outer.pop_back();
            i += best.reps * best.period;
            out.push_back(std::move(best));
        } else {
            ++i;
        }
    }
    return out;
}

// Micro-ops emitted for [lo, hi) with `runs` rolled.
size_t emitted_ops(const std::vector<Run> &runs, size_t lo, size_t hi)
{
    size_t n = hi - lo;
    for (const Run &r : runs) n = n - r.reps * r.period + emitted_ops(r.inner, r.start, r.start + r.period);
    return n;
}

bool analyze(const SchedProgram &p, const JitLimits &lim, Graph &g, std::string &why)
{
    g.lim = &lim;
    g.D = assemble_device(p, 8, g.entry);
    const size_t nv = g.entry.size();
    if (nv == 0) {
        why = "empty schedule";
        return false;
    }
    g.seen.assign(nv, 0);
    g.used_reg.assign(p.nregs + 1, 0);
    g.used_reg[p.in_reg] = 1;
    std::vector<std::vector<uint32_t>> succ(nv);
    std::deque<uint32_t> work{0};
    g.seen[0] = 1;
    auto reach = [&](uint32_t from, uint64_t v) -> bool {
        if (v >= nv) return false;
        succ[from].push_back((uint32_t)v);
        if (!g.seen[v]) {
            g.seen[v] = 1;
            work.push_back((uint32_t)v);
        }
        return true;
    };
    while (!work.empty()) {
        const uint32_t v = work.front();
        work.pop_front();
        if (++g.nreach > lim.max_variants) {
            why = "too many superblock variants for the native tier";
            return false;
        }
        for (size_t pc = g.entry[v];; ++pc) {
            if (pc >= g.D.size()) {
                why = "superblock runs off the code";
                return false;
            }
            if (++g.ndops > lim.max_scan) {
                why = "schedule too large for the native tier";
                return false;
            }
            const DOp &I = g.D[pc];
            auto use = [&](uint32_t off) {
                if (off / 8 < g.used_reg.size()) g.used_reg[off / 8] = 1;
            };
            bool leave = false, ok = true;
            switch (I.op) {
            case U_MOV: case U_ADDI: case U_RSUBI: use(I.a); use(I.d); break;
            case U_ADD: case U_SUB: use(I.a); use(I.b); use(I.d); break;
            case U_LI: case U_LD: use(I.d); break;
            case U_ST: use(I.a); break;
            case U_STI: break;
            case U_STX: use(I.a); use(I.b); break;
            case U_LDX: use(I.d); use(I.b); break;
            case U_OVF: if (I.fl & UF_OUTREG) use(I.a); use(I.b); break;
            case U_BRX: use(I.a); ok = reach(v, (uint64_t)I.imm); break;
            case U_JUMP: ok = reach(v, (uint64_t)I.imm); leave = true; break;
            case U_BR:
                use(I.a);
                ok = reach(v, (uint32_t)(uint64_t)I.imm) && reach(v, (uint64_t)I.imm >> 32);
                leave = true;
                break;
            case U_JRO:
                use(I.a);
                for (uint64_t t = 0; t <= I.b && ok; ++t) {
                    const uint64_t j = (uint64_t)I.imm + t;
                    ok = j < p.jtab.size() && reach(v, p.jtab[j]);
                }
                leave = true;
                break;
            case U_END: if (I.fl & UF_OUTREG) use(I.a); leave = true; break;
            case U_YIELD: // sessions: a call ends; the next one starts at variant lo32(imm)
                if (I.fl & UF_OUTREG) use(I.a);
                ok = reach(v, (uint32_t)(uint64_t)I.imm);
                leave = true;
                break;
            case U_HANDOFF: leave = true; break; // sessions: the interpreter goes on from this entry
            case U_GUARD: ok = reach(v, (uint64_t)I.imm); break;
            case U_ROUND_END: if (I.fl & UF_OUTREG) use(I.a); break;
            default: ok = false;
            }
            if (!ok) {
                why = "malformed schedule";
                return false;
            }
            if (leave) break;
        }
    }
    for (uint32_t r = 0; r < g.used_reg.size(); ++r)
        if (g.used_reg[r] && r >= p.nregs) {
            why = "register out of range";
            return false;
        }
    // roll repeating stretches; the emitted size is what the limit applies to
    // (acyclic: the GPU kernel holds only the variants reachable without
    // taking a guard -- see emit_stream)
    std::vector<char> counted = g.seen;
    if (!g.cyclic) {
        counted.assign(nv, 0);
        std::deque<uint32_t> q{0};
        counted[0] = 1;
        while (!q.empty()) {
            const uint32_t v = q.front();
            q.pop_front();
            for (uint32_t w : succ[v])
                if (!(v & 1u) && w == v + 1 && g.D[g.entry[v]].op == U_GUARD) continue; // the guard edge
                else if (!counted[w]) counted[w] = 1, q.push_back(w);
        }
    }
    g.runs.assign(nv, {});
    g.ndops = 0;
    for (uint32_t v = 0; v < nv; ++v) {
        if (!g.seen[v]) continue;
        size_t lo = g.entry[v], hi = lo;
        if (g.D[lo].op == U_GUARD) ++lo, ++hi;
        while (body_op(g.D[hi].op)) ++hi;
        std::vector<const Run *> outer;
        g.runs[v] = find_runs(g.D, lo, hi, outer);
        if (counted[v]) g.ndops += (lo - g.entry[v]) + emitted_ops(g.runs[v], lo, hi) + 1;
    }
    if (g.ndops > lim.max_dops) {
        why = "schedule too large for the native tier";
        return false;
    }
    // cycle detection over reachable variants (iterative DFS, colours 0/1/2)
    std::vector<uint8_t> col(nv, 0);
    std::vector<std::pair<uint32_t, size_t>> st{{0u, 0}};
    col[0] = 1;
    while (!st.empty() && !g.cyclic) {
        auto &[v, k] = st.back();
        if (k < succ[v].size()) {
            const uint32_t w = succ[v][k++];
            if (col[w] == 1) g.cyclic = true;
            else if (col[w] == 0) {
                col[w] = 1;
                st.push_back({w, 0});
            }
        } else {
            col[v] = 2;
            st.pop_back();
        }
    }
    g.succ = std::move(succ);
    return true;
}

// The reachable variants in reverse postorder from variant 0: every edge
// goes forward except the back edges of cycles (a JRO's backward arms, a
// lane's wrap to its program's start) and self-loops.
std::vector<uint32_t> forward_order(const Graph &g)
{
    const size_t nv = g.entry.size();
    std::vector<std::vector<uint32_t>> succ = g.succ;
    for (auto &l : succ) std::sort(l.begin(), l.end(), std::greater<uint32_t>());
    std::vector<uint8_t> col(nv, 0);
    std::vector<uint32_t> post;
    std::vector<std::pair<uint32_t, size_t>> st{{0u, 0}};
    col[0] = 1;
    while (!st.empty()) {
        auto &[v, k] = st.back();
        if (k < succ[v].size()) {
            // successors in descending id order, so that the lower ids (a
            // fast variant before its checked one) come first in the result
            const uint32_t w = succ[v][k++];
            if (!col[w]) {
                col[w] = 1;
                st.push_back({w, 0});
            }
        } else {
            post.push_back(v);
            st.pop_back();
        }
    }
    return std::vector<uint32_t>(post.rbegin(), post.rend());
}

// Registers whose high 32 bits no reachable op ever reads.  ACC and BAK are
// int64 (program.go:27-28) and every hop truncates to int32 (program.go:498,
// 516, 561), so a register that only ever feeds hops -- stack slots, the
// /compute output, port hand-offs to sext32 uses -- or other such registers
// through ADD/SUB/MOV (whose low 32 bits depend on their operands' low 32
// bits only) can be computed in 32 bits with identical results.  The high
// bits are read by BR/BRX conditions and JRO operands without UF_TA (the
// full int64 ACC decides, program.go:315-363), by dynamic-stack depth
// operands (STX/LDX/OVF b), and by any op writing a register that needs
// them.  A backward fixpoint over the reachable ops, flow-insensitive.
// C4's pipeline then runs its `sum = 3 * sum + v` chains as 32-bit adds
// instead of 64-bit ones (half the VALU work, and the same code from either
// hiprtc).  Stream shape only: the machine shape's loop phases keep int64.
void narrow_regs(Graph &g)
{
    const size_t R = g.used_reg.size();
    std::vector<char> wide(R, 0);
    std::vector<const DOp *> ops;
    for (uint32_t v = 0; v < g.entry.size(); ++v) {
        if (!g.seen[v]) continue;
        for (size_t pc = g.entry[v];; ++pc) {
            const DOp &I = g.D[pc];
            ops.push_back(&I);
            if (I.op == U_JUMP || I.op == U_BR || I.op == U_JRO || I.op == U_END) break;
        }
    }
    auto mark = [&](uint32_t off) {
        const uint32_t r = off / 8;
        if (r < R && !wide[r]) { wide[r] = 1; return true; }
        return false;
    };
    for (const DOp *I : ops) {
        switch (I->op) {
        case U_BR: case U_BRX: case U_JRO: if (!(I->fl & UF_TA)) mark(I->a); break;
        case U_STX: case U_LDX: case U_OVF: mark(I->b); break;
        default: break;
        }
    }
    for (bool changed = true; changed;) {
        changed = false;
        for (const DOp *I : ops) {
            if (!(I->d / 8 < R && wide[I->d / 8])) continue;
            switch (I->op) {
            case U_MOV: case U_ADDI: case U_RSUBI: if (!(I->fl & UF_TA)) changed |= mark(I->a); break;
            case U_ADD: case U_SUB:
                if (!(I->fl & UF_TA)) changed |= mark(I->a);
                if (!(I->fl & UF_TB)) changed |= mark(I->b);
                break;
            default: break;
            }
        }
    }
    g.narrow.assign(R, 0);
    for (size_t r = 0; r < R; ++r) g.narrow[r] = g.used_reg[r] && !wide[r];
}

// Micro-op emission shared by both shapes.  `R` prefixes register names
// ("r" for locals of the stream lane function, "L.r" for the machine's lane
// state); `exit_*` print the shape's form of each superblock exit.
struct OpWriter {
    Emitter &e;
    const SchedProgram &p;
    const char *R;

    std::string operand(uint32_t off, bool trunc) const
    {
        char b[64];
        if (trunc)
            snprintf(b, sizeof b, "((int64_t)(int32_t)%s%u)", R, off / 8);
        else
            snprintf(b, sizeof b, "%s%u", R, off / 8);
        return b;
    }

    std::string result(const DOp &I) const
    {
        if (I.fl & UF_OUTREG) return "(int32_t)" + operand(I.a, I.fl & UF_TA);
        char b[48];
        snprintf(b, sizeof b, "(int32_t)%" PRId32, (int32_t)I.imm);
        return b;
    }

    std::string cond(const DOp &I) const
    {
        static const char *const cmp[4] = {"== 0", "!= 0", "> 0", "< 0"};
        return "(" + operand(I.a, I.fl & UF_TA) + " " + cmp[(I.fl >> UF_COND_SHIFT) & 3u] + ")";
    }

    // Data micro-ops; returns false for an exit / control op.  `slot`
    // overrides the slot number of ST/LD/STI (an expression in a rolled loop).
    bool data(const DOp &I, const char *slot = nullptr) const
    {
        const std::string A = operand(I.a, I.fl & UF_TA), B = operand(I.b, I.fl & UF_TB);
        const uint32_t d = I.d / 8;
        char sb[64];
        if (!slot) {
            snprintf(sb, sizeof sb, "%uu", I.op == U_STI ? I.d : (uint32_t)I.imm);
            slot = sb;
        }
        switch (I.op) {
        case U_MOV: e.line("    %s%u = %s;", R, d, A.c_str()); return true;
        case U_LI: e.line("    %s%u = (int64_t)%s;", R, d, u64lit(I.imm).c_str()); return true;
        case U_ADD: e.line("    %s%u = (int64_t)((uint64_t)%s + (uint64_t)%s);", R, d, A.c_str(), B.c_str()); return true;
        case U_SUB: e.line("    %s%u = (int64_t)((uint64_t)%s - (uint64_t)%s);", R, d, A.c_str(), B.c_str()); return true;
        case U_ADDI: e.line("    %s%u = (int64_t)((uint64_t)%s + %s);", R, d, A.c_str(), u64lit(I.imm).c_str()); return true;
        case U_RSUBI: e.line("    %s%u = (int64_t)(%s - (uint64_t)%s);", R, d, u64lit(I.imm).c_str(), A.c_str()); return true;
        case U_ST: e.line("    MK_SLOT_ST(slots, sstride, %s, (int32_t)%s);", slot, A.c_str()); return true;
        case U_STI:
            e.line("    MK_SLOT_ST(slots, sstride, %s, (int32_t)%" PRId32 ");", slot, (int32_t)I.imm);
            return true;
        case U_LD: e.line("    %s%u = (int64_t)MK_SLOT_LD(slots, sstride, %s);", R, d, slot); return true;
        // dynamic stacks: slot imm + index register (a per-lane slot number)
        case U_STX:
            e.line("    MK_SLOT_STX(slots, sstride, (uint32_t)(%uu + (uint32_t)%s), (int32_t)%s);", (uint32_t)I.imm,
                   operand(I.b, false).c_str(), A.c_str());
            return true;
        case U_LDX:
            e.line("    %s%u = (int64_t)MK_SLOT_LDX(slots, sstride, (uint32_t)(%uu + (uint32_t)%s));", R, d,
                   (uint32_t)I.imm, operand(I.b, false).c_str());
            return true;
        default: return false;
        }
    }

    // OVF: a PUSH onto a dynamic stack at its capacity ends the lane
    std::string ovf_cond(const DOp &I) const { return "((uint64_t)" + operand(I.b, false) + " >= " + std::to_string((uint64_t)I.imm >> 32) + "ull)"; }
    std::string ovf_result(const DOp &I) const
    {
        if (I.fl & UF_OUTREG) return "(int32_t)" + operand(I.a, I.fl & UF_TA);
        char b[48];
        snprintf(b, sizeof b, "(int32_t)%" PRId32, (int32_t)(uint32_t)(uint64_t)I.imm);
        return b;
    }

    // t = IntClamp(ip + A, 0, len-1) with an int64 wrapping add (program.go:354,362)
    void jro_target(const DOp &I) const
    {
        e.line("        int64_t t = (int64_t)((uint64_t)%uu + (uint64_t)%s);", I.d, operand(I.a, I.fl & UF_TA).c_str());
        e.line("        t = t > (int64_t)%u ? (int64_t)%u : t;", I.b, I.b);
        e.line("        t = t < 0 ? 0 : t;");
    }
};

// A rolled loop whose body only reads stack slots (a run of POPs: LD ops, no
// ST) is software-pipelined: while one block of U iterations uses its
// popped values, the slots of the next block are already being read, so a
// wave keeps ~lim.prefetch spill reads in flight instead of draining its
// loads at every unrolled step (C4's pop loops are a serial ACC chain over
// the popped values).  Two register sets (A, B) alternate, so no value is
// copied while its load is in flight (a copy would need the load's wait).
// Reading ahead is safe because nothing in the loop writes a slot.  Returns
// false (nothing emitted) for other runs.
template <class Expr, class RoundEnd>
bool emit_prefetched_run(const OpWriter &w, const Graph &g, const Run &r, std::vector<const Run *> &outer,
                         const Expr &expr, RoundEnd &round_end)
{
    if (!r.inner.empty()) return false;
    const size_t depth = g.lim->prefetch; // loads in flight, 0 = off (MK_JIT_PREFETCH)
    if (!depth) return false;
    std::vector<size_t> lds;
    for (size_t pc = r.start; pc < r.start + r.period; ++pc) {
        const DOp &I = g.D[pc];
        if (I.op == U_ST || I.op == U_STI || I.op == U_STX || I.op == U_OVF || I.op == U_BRX) return false;
        if (I.op == U_LD) lds.push_back(pc);
    }
    if (lds.empty()) return false;
    const size_t U = std::max<size_t>(2, depth / lds.size());
    if (r.reps < 4 * U) return false;
    const size_t D = outer.size(), jn = r.reps - r.reps % (2 * U);
    Emitter &e = w.e;
    outer.push_back(&r);
    // set `set` <- block starting at iteration `it`; an index past the loop
    // is clamped to its last iteration (the final read-ahead re-reads a slot
    // of the loop instead of leaving its range)
    auto load = [&](char set, const std::string &it) {
        for (size_t a = 0; a < lds.size(); ++a)
            for (size_t k = 0; k < U; ++k)
                e.line("    { const uint32_t j%zu = %s + %zuu < %zuu ? %s + %zuu : %zuu; "
                       "%c%zu_%zu_%zu = MK_SLOT_LD(slots, sstride, %s); }",
                       D, it.c_str(), k, r.reps - 1, it.c_str(), k, r.reps - 1, set, D, a, k,
                       expr(lds[a], advancing(g.D[lds[a]])).c_str());
        // keeps the read-ahead here: LLVM otherwise sinks each load to its use
        e.line("    __asm__ volatile(\"\" ::: \"memory\");");
    };
    auto body = [&](char set, const std::string &it) {
        for (size_t k = 0; k < U; ++k) {
            e.line("    { const uint32_t j%zu = %s + %zuu; (void)j%zu;", D, it.c_str(), k, D);
            for (size_t pc = r.start, a = 0; pc < r.start + r.period; ++pc) {
                const DOp &I = g.D[pc];
                if (I.op == U_LD) e.line("    %s%u = (int64_t)%c%zu_%zu_%zu;", w.R, I.d / 8, set, D, a++, k);
                else if (I.op == U_ROUND_END) round_end(I, ("(uint64_t)(" + expr(pc, I.inc) + ")").c_str(), pc);
                else w.data(I);
            }
            e.line("    }");
        }
    };
    const std::string jb = "jb" + std::to_string(D);
    e.line("    {");
    for (char set : {'A', 'B'})
        for (size_t a = 0; a < lds.size(); ++a)
            for (size_t k = 0; k < U; ++k) e.line("    int32_t %c%zu_%zu_%zu;", set, D, a, k);
    load('A', "0u");
    e.line("    for (uint32_t %s = 0; %s < %zuu; %s += %zuu) {", jb.c_str(), jb.c_str(), jn, jb.c_str(), 2 * U);
    load('B', jb + " + " + std::to_string(U) + "u");
    body('A', jb);
    load('A', jb + " + " + std::to_string(2 * U) + "u");
    body('B', jb + " + " + std::to_string(U) + "u");
    e.line("    }");
    if (jn < r.reps) { // the last reps % 2U iterations, unpipelined
        e.line("    for (uint32_t j%zu = %zuu; j%zu < %zuu; ++j%zu) {", D, jn, D, r.reps, D);
        for (size_t pc = r.start; pc < r.start + r.period; ++pc) {
            const DOp &I = g.D[pc];
            if (slot_op(I)) w.data(I, expr(pc, advancing(I)).c_str());
            else if (I.op == U_ROUND_END) round_end(I, ("(uint64_t)(" + expr(pc, I.inc) + ")").c_str(), pc);
            else w.data(I);
        }
        e.line("    }");
    }
    e.line("    }");
    outer.pop_back();
    return true;
}

// Emits the body [lo, hi) of a variant -- data ops and ROUND_END markers --
// rolling `runs` into nested for loops (loop variables j0, j1, ...); an
// op's slot or step count is its value in the first copy plus, per
// enclosing loop, that loop's variable times the op's advance.
// `round_end(I, inc, pc)` prints a ROUND_END (at pc of the first copy) whose
// step count is the expression `inc`.
template <class RoundEnd>
void emit_rolled(const OpWriter &w, const Graph &g, const std::vector<Run> &runs, size_t lo, size_t hi,
                 std::vector<const Run *> &outer, RoundEnd &round_end)
{
    size_t ri = 0;
    auto expr = [&](size_t pc, int64_t base) {
        std::string x = std::to_string(base) + "ll";
        for (size_t L = 0; L < outer.size(); ++L) {
            const int64_t d = outer[L]->delta[pc - outer[L]->start];
            if (d) x += " + (int64_t)j" + std::to_string(L) + " * " + std::to_string(d) + "ll";
        }
        return x;
    };
    for (size_t pc = lo; pc < hi;) {
        if (ri < runs.size() && runs[ri].start == pc) {
            const Run &r = runs[ri++];
            if (emit_prefetched_run(w, g, r, outer, expr, round_end)) {
                pc += r.reps * r.period;
                continue;
            }
            w.e.line("    for (uint32_t j%zu = 0; j%zu < %zuu; ++j%zu) {", outer.size(), outer.size(), r.reps,
                     outer.size());
            outer.push_back(&r);
            emit_rolled(w, g, r.inner, r.start, r.start + r.period, outer, round_end);
            outer.pop_back();
            w.e.line("    }");
            pc += r.reps * r.period;
            continue;
        }
        const DOp &I = g.D[pc];
        if (slot_op(I)) {
            w.data(I, expr(pc, advancing(I)).c_str());
        } else if (I.op == U_ROUND_END || I.op == U_OVF || I.op == U_BRX) { // in-line ends / exits: the shape's callback
            round_end(I, ("(uint64_t)(" + expr(pc, I.inc) + ")").c_str(), pc);
        } else {
            w.data(I);
        }
        ++pc;
    }
}

template <class RoundEnd>
void emit_body(const OpWriter &w, const Graph &g, uint32_t v, size_t lo, size_t hi, RoundEnd round_end)
{
    std::vector<const Run *> outer;
    emit_rolled(w, g, g.runs[v], lo, hi, outer, round_end);
}

// ---- budget exits of checked variants ----------------------------------------
// A checked variant is entered only through its fast variant's GUARD, which
// fires when steps + (largest round-end count inside) >= budget: every lane
// in it therefore ends at a round end inside it -- the first round end R
// whose count inc_R >= budget - steps -- with status BUDGET (plus HAS_OUTPUT
// if an OUT completed by round R), steps + inc_R, and the /compute output as
// of round R.  The exit op is never reached.
//
// So instead of a test and an early exit per round end (a deep pipeline has
// thousands: C4 d64's checked variant alone had 5,643, and that CFG took
// hiprtc minutes), the checked variant runs its whole body -- the same data
// ops as the fast variant; stack-slot writes past R are harmless because the
// lane ends -- and then looks R up in the list of its round ends, compressed
// into arithmetic runs of counts with one status each.  The output value is
// read once, at the last round end that has one: the schedule compiler sets
// the output location only at the first OUT (tis_sched.cpp OUTL), so every
// round end with HAS_OUTPUT sees the same value.
struct ReSeg {
    int64_t first = 0, step = 1, last = 0;
    uint32_t st = 0;
};

struct RoundEnds {
    std::vector<ReSeg> segs;
    size_t snap_pc = SIZE_MAX; // pc (first copy) of the last round end with an output
};

void collect_round_ends(const Graph &g, const std::vector<Run> &runs, size_t lo, size_t hi,
                        std::vector<std::pair<const Run *, int64_t>> &outer,
                        std::vector<std::pair<int64_t, uint32_t>> &out, size_t &snap_pc)
{
    size_t ri = 0;
    for (size_t pc = lo; pc < hi;) {
        if (ri < runs.size() && runs[ri].start == pc) {
            const Run &r = runs[ri++];
            for (size_t j = 0; j < r.reps; ++j) {
                outer.push_back({&r, (int64_t)j});
                collect_round_ends(g, r.inner, r.start, r.start + r.period, outer, out, snap_pc);
                outer.pop_back();
            }
            pc += r.reps * r.period;
            continue;
        }
        const DOp &I = g.D[pc];
        if (I.op == U_ROUND_END) {
            int64_t inc = I.inc;
            for (const auto &[o, j] : outer) inc += j * o->delta[pc - o->start];
            out.push_back({inc, (uint32_t)I.d});
            if (I.d & MK_ST_HAS_OUTPUT) snap_pc = pc;
        }
        ++pc;
    }
}

RoundEnds round_ends(const Graph &g, uint32_t v, size_t lo, size_t hi)
{
    RoundEnds re;
    std::vector<std::pair<const Run *, int64_t>> outer;
    std::vector<std::pair<int64_t, uint32_t>> all;
    collect_round_ends(g, g.runs[v], lo, hi, outer, all, re.snap_pc);
    // counts never decrease; of equal counts only the first can be R
    std::vector<std::pair<int64_t, uint32_t>> u;
    for (const auto &x : all)
        if (u.empty() || x.first > u.back().first) u.push_back(x);
    for (size_t i = 0; i < u.size();) {
        ReSeg s;
        s.first = s.last = u[i].first;
        s.st = u[i].second;
        size_t k = i + 1;
        if (k < u.size() && u[k].second == s.st) {
            s.step = u[k].first - s.first;
            while (k < u.size() && u[k].second == s.st && u[k].first - s.last == s.step) s.last = u[k++].first;
        }
        re.segs.push_back(s);
        i = k;
    }
    return re;
}

// The lookup after a checked variant's body: sets `inc_` and `st_` (locals
// declared here) for need = budget - steps (`steps` is the lane's count
// expression at variant entry).
void emit_budget_exit(Emitter &e, Emitter &tab, const RoundEnds &re, uint32_t v, const char *steps)
{
    e.line("    const int64_t need_ = (int64_t)budget - (int64_t)%s;", steps);
    e.line("    uint32_t inc_, st_;");
    auto one = [&](const ReSeg &s, const char *pre) {
        if (s.first == s.last)
            e.line("    %s{ inc_ = %lldu; st_ = %uu; }", pre, (long long)s.first, s.st);
        else
            e.line("    %s{ inc_ = need_ <= %lldll ? %lldu : (uint32_t)(%lldll + (need_ - %lldll + %lldll) / %lldll * %lldll); "
                   "st_ = %uu; }",
                   pre, (long long)s.first, (long long)s.first, (long long)s.first, (long long)s.first,
                   (long long)(s.step - 1), (long long)s.step, (long long)s.step, s.st);
    };
    const size_t n = re.segs.size();
    if (n <= 8) {
        for (size_t i = 0; i + 1 < n; ++i) {
            char pre[64];
            snprintf(pre, sizeof pre, "%sif (need_ <= %lldll) ", i ? "else " : "", (long long)re.segs[i].last);
            one(re.segs[i], pre);
        }
        one(re.segs[n - 1], n > 1 ? "else " : "");
        return;
    }
    // many segments: binary search over a table {last, first, step, st}
    std::string t;
    for (const ReSeg &s : re.segs) {
        char b[96];
        snprintf(b, sizeof b, "%lldu,%lldu,%lldu,%uu,", (long long)s.last, (long long)s.first, (long long)s.step, s.st);
        t += b;
    }
    tab.line("MK_CTABLE uint32_t mk_re%u[] = {%s};", v, t.c_str());
    e.line("    {");
    e.line("    const uint32_t *re_ = mk_re%u;", v);
    e.line("    uint32_t lo_ = 0u, hi_ = %zuu;", n - 1);
    e.line("    while (lo_ < hi_) {");
    e.line("        const uint32_t m_ = (lo_ + hi_) >> 1;");
    e.line("        if (need_ <= (int64_t)re_[4u * m_]) hi_ = m_; else lo_ = m_ + 1u;");
    e.line("    }");
    e.line("    const int64_t f_ = re_[4u * lo_ + 1u], s_ = re_[4u * lo_ + 2u];");
    e.line("    inc_ = need_ <= f_ ? (uint32_t)f_ : (uint32_t)(f_ + (need_ - f_ + s_ - 1) / s_ * s_);");
    e.line("    st_ = re_[4u * lo_ + 3u];");
    e.line("    }");
}

// Whether [lo, hi) holds an OVF or a BRX (a checked variant with one cannot
// use the budget-exit lookup: a lane may end or leave there before its
// round end).
bool has_inline_exit(const Graph &g, size_t lo, size_t hi)
{
    for (size_t pc = lo; pc < hi; ++pc)
        if (g.D[pc].op == U_OVF || g.D[pc].op == U_BRX) return true;
    return false;
}

// In-line ends of a body, in program order: OVF (capacity), BRX (a side
// exit to another variant) and, in checked variants that cannot use the
// lookup, ROUND_END (budget).  `L` prefixes the lane state ("" or "L."),
// `fin` is the statement that ends the lane, `go` (a printf format of the
// target variant) the one that continues it elsewhere.
void emit_inline_end(const OpWriter &w, const DOp &I, const char *inc, const char *L, const char *fin,
                     const char *go)
{
    if (I.op == U_BRX) {
        w.e.line("    if %s {", w.cond(I).c_str());
        w.e.line("        %ssteps += %uu;", L, I.inc);
        char b[96];
        snprintf(b, sizeof b, go, (uint32_t)I.imm);
        w.e.line("        %s", b);
        w.e.line("    }");
        return;
    }
    if (I.op == U_OVF) {
        w.e.line("    if %s {", w.ovf_cond(I).c_str());
        w.e.line("        %ssteps += %uu;", L, I.inc);
        w.e.line("        %soutv = %s;", L, w.ovf_result(I).c_str());
    } else {
        w.e.line("    if ((uint64_t)%ssteps + %s >= (uint64_t)budget) {", L, inc);
        w.e.line("        %ssteps += (uint32_t)%s;", L, inc);
        w.e.line("        %soutv = %s;", L, w.result(I).c_str());
    }
    w.e.line("        %sst = %uu;", L, I.d);
    w.e.line("        %s", fin);
    w.e.line("    }");
}

// [lo, hi) of variant v's body: after its GUARD, up to its exit op.
void body_range(const Graph &g, uint32_t v, size_t &lo, size_t &hi)
{
    lo = g.entry[v];
    if (g.D[lo].op == U_GUARD) ++lo;
    hi = lo;
    while (body_op(g.D[hi].op)) ++hi;
}

// ---- stream shape: straight-line lane function ------------------------------

// Longest path, in retired instructions, from variant 0 through fast
// variants only (the guard never fires on it); the graph is acyclic here.
uint64_t max_fast_steps(const SchedProgram &p, const Graph &g)
{
    std::vector<int64_t> memo(g.entry.size(), -1);
    std::vector<uint32_t> stack{0u};
    // iterative post-order DFS
    std::vector<uint8_t> state(g.entry.size(), 0);
    // successors of v with the steps retired on the way to each (a BRX leaves
    // mid-body with its own count)
    std::vector<uint64_t> sinc;
    auto exits = [&](uint32_t v, std::vector<uint32_t> &succ) -> uint64_t {
        succ.clear();
        sinc.clear();
        for (size_t pc = g.entry[v];; ++pc) {
            const DOp &I = g.D[pc];
            const size_t n0 = succ.size();
            switch (I.op) {
            case U_BRX: succ.push_back((uint32_t)I.imm); sinc.push_back(I.inc); continue;
            case U_JUMP: succ.push_back((uint32_t)I.imm); break;
            case U_BR:
                succ.push_back((uint32_t)(uint64_t)I.imm);
                succ.push_back((uint32_t)((uint64_t)I.imm >> 32));
                break;
            case U_JRO:
                for (uint64_t t = 0; t <= I.b; ++t) succ.push_back(p.jtab[(size_t)I.imm + t]);
                break;
            case U_END: return I.inc;
            default: continue;
            }
            while (sinc.size() < succ.size()) sinc.push_back(I.inc);
            (void)n0;
            return I.inc;
        }
    };
    std::vector<uint32_t> succ;
    while (!stack.empty()) {
        const uint32_t v = stack.back();
        if (state[v] == 0) {
            state[v] = 1;
            exits(v, succ);
            for (uint32_t w : succ)
                if (state[w] == 0) stack.push_back(w);
            continue;
        }
        stack.pop_back();
        if (state[v] == 2) continue;
        const uint64_t inc = exits(v, succ);
        int64_t best = (int64_t)inc; // END (or no successor)
        for (size_t k = 0; k < succ.size(); ++k) best = std::max<int64_t>(best, (int64_t)sinc[k] + memo[succ[k]]);
        memo[v] = best;
        state[v] = 2;
    }
    return (uint64_t)memo[0];
}

// The lane function.  `unguarded`: the variant for launches whose budget
// exceeds every path (max_fast_steps) -- no GUARD tests, no checked variants.
void emit_stream_lane(const SchedProgram &p, const Graph &g, Emitter &e, const char *name, bool unguarded)
{
    OpWriter w{e, p, "r"};
    const size_t nv = g.entry.size();
    std::vector<char> live(nv, 0);
    if (unguarded) {
        std::deque<uint32_t> q{0};
        live[0] = 1;
        auto add = [&](uint32_t v) {
            if (v < nv && !live[v]) {
                live[v] = 1;
                q.push_back(v);
            }
        };
        while (!q.empty()) {
            const uint32_t v = q.front();
            q.pop_front();
            for (size_t pc = g.entry[v];; ++pc) {
                const DOp &I = g.D[pc];
                if (I.op == U_BRX) { add((uint32_t)I.imm); continue; }
                if (I.op == U_JUMP) { add((uint32_t)I.imm); break; }
                if (I.op == U_BR) { add((uint32_t)(uint64_t)I.imm); add((uint32_t)((uint64_t)I.imm >> 32)); break; }
                if (I.op == U_JRO) {
                    for (uint64_t t = 0; t <= I.b; ++t) add(p.jtab[(size_t)I.imm + t]);
                    break;
                }
                if (I.op == U_END) break;
            }
        }
    } else {
        live = g.seen;
    }
    Emitter tab; // budget-exit tables of checked variants (before the function)
    const size_t fn_start = e.s.size();
    e.line("MK_FN int32_t %s(int64_t in, uint32_t budget, int32_t *__restrict__ slots, uint64_t sstride,", name);
    e.line("                      uint32_t *steps_out, uint32_t *status_out)");
    e.line("{");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    %s r%u = 0;", r < g.narrow.size() && g.narrow[r] ? "uint32_t" : "int64_t", r);
    e.line("    r%u = (int64_t)(int32_t)in;", p.in_reg);
    e.line("    uint32_t steps = 0, st = 0;");
    e.line("    int32_t outv = 0;");
    e.line("    (void)slots; (void)sstride; (void)budget;");
    for (uint32_t v = 0; v < nv; ++v) {
        if (!live[v]) continue;
        e.line("V%u:", v);
        const DOp &G = g.D[g.entry[v]];
        if (G.op == U_GUARD && !unguarded)
            e.line("    if ((uint64_t)steps + %uu >= (uint64_t)budget) goto V%u;", G.inc, (uint32_t)G.imm);
        size_t lo, hi;
        body_range(g, v, lo, hi);
        const RoundEnds re = round_ends(g, v, lo, hi);
        const bool ovf = has_inline_exit(g, lo, hi);
        if (!re.segs.empty() && !ovf) { // checked variant: always ends at a round end (emit_budget_exit)
            e.line("    {");
            e.line("    int32_t mk_o = 0;");
            emit_body(w, g, v, lo, hi, [&](const DOp &I, const char *, size_t pc) {
                if (pc == re.snap_pc) e.line("    mk_o = %s;", w.result(I).c_str());
            });
            emit_budget_exit(e, tab, re, v, "steps");
            e.line("    steps += inc_;");
            e.line("    st = st_;");
            e.line("    outv = (st_ & %uu) ? mk_o : 0;", (unsigned)MK_ST_HAS_OUTPUT);
            e.line("    (void)mk_o;");
            e.line("    goto done;");
            e.line("    }");
            continue;
        }
        emit_body(w, g, v, lo, hi, [&](const DOp &I, const char *inc, size_t) {
            emit_inline_end(w, I, inc, "", "goto done;", "goto V%u;");
        });
        const DOp &I = g.D[hi];
        switch (I.op) {
        case U_JUMP:
            e.line("    steps += %uu;", I.inc);
            e.line("    goto V%u;", (uint32_t)I.imm);
            break;
        case U_BR:
            e.line("    steps += %uu;", I.inc);
            e.line("    if %s goto V%u;", w.cond(I).c_str(), (uint32_t)(uint64_t)I.imm);
            e.line("    goto V%u;", (uint32_t)((uint64_t)I.imm >> 32));
            break;
        case U_JRO: {
            e.line("    steps += %uu;", I.inc);
            e.line("    {");
            w.jro_target(I);
            e.line("        switch (t) {");
            const uint32_t last = p.jtab[(size_t)I.imm + I.b];
            for (uint32_t t = 0; t < I.b; ++t) {
                const uint32_t tgt = p.jtab[(size_t)I.imm + t];
                if (tgt != last) e.line("        case %u: goto V%u;", t, tgt);
            }
            e.line("        default: goto V%u;", last);
            e.line("        }");
            e.line("    }");
            break;
        }
        case U_END:
            e.line("    steps += %uu;", I.inc);
            e.line("    outv = %s;", w.result(I).c_str());
            e.line("    st = %uu;", I.d);
            e.line("    goto done;");
            break;
        default: break;
        }
    }
    e.line("done:");
    e.line("    *steps_out = steps;");
    e.line("    *status_out = st;");
    e.line("    return outv;");
    e.line("}");
    e.s.insert(fn_start, tab.s);
}

// The kernel runs only launches whose budget exceeds every path
// (MK_MAX_STEPS): its lane function has no guards and no checked variants.
// The guarded lane (MK_LANE_CHECKED) is for the CPU tests; the executor
// gives launches with a smaller budget to tier 2.
// Stream lanes with more than lim.heavy_ops micro-ops run in the heavy kernel.
// How the heavy kernel reaches its LDS slots: slot s of lane l at word
// s * 64 + l.  LLVM may forward a store to the load that pops it and keep
// the value in registers (nothing else touches the wave's LDS).  (Volatile
// accesses and quad-interleaved slots were measured and lost: round 2-3,
// DESIGN section 4b; removed in round 6.)
void emit_lds_access(Emitter &e, const JitLimits &lim)
{
    (void)lim;
    e.line("#define MK_LDS_SLOTS mk_lds_slots");
    e.line("#define MK_LDS_IX(s) ((uint32_t)(s) * 64u + (threadIdx.x & 63u))");
}

void emit_stream(const SchedProgram &p, const Graph &g, Emitter &e, uint64_t max_steps, bool checked)
{
    e.line("// generated from a compiled schedule: %zu variants reachable, %zu micro-ops, acyclic", g.nreach, g.ndops);
    e.line("#define MK_JIT_MACHINE 0");
    e.line("#ifndef MK_CTABLE");
    e.line("#define MK_CTABLE static const");
    e.line("#endif");
    e.line("#define MK_MAX_STEPS %lluull", (unsigned long long)max_steps);
    e.line("#define MK_NSLOTS %uu", p.nslots);
    // MK_JIT_SLOT_LAYOUT=blocked|lane overrides the choice (tests, tuning)
    const bool blocked = g.lim->slot_layout >= 0 ? g.lim->slot_layout == 1 : p.nslots <= kJitWaveBlockedSlots;
    e.line("#define MK_SLOTS_WAVE_BLOCKED %d", blocked ? 1 : 0);
    const uint32_t nl = jit_lds_slot_count(p.nslots, g.ndops > g.lim->heavy_ops, *g.lim);
    if (nl && nl < p.nslots) {
        // Heavy kernel, slots split: the first nl slots of a lane in LDS (as
        // below), the rest in the wave's HBM block (buffer ops, as after).
        // A slot number is wave-uniform for ordinary stacks, so the test is a
        // scalar branch (per lane for dynamic stacks).
        e.line("#ifndef MK_LANE_CHECKED");
        e.line("#define MK_SLOTS_BUFFER 1");
        e.line("#define MK_SLOTS_LDS_N %uu", nl);
        e.line("#define MK_HBM_NSLOTS (MK_NSLOTS - MK_SLOTS_LDS_N)");
        e.line("__shared__ int32_t mk_lds_slots[MK_SLOTS_LDS_N * 64u];");
        emit_lds_access(e, *g.lim);
        e.line("MK_FN __amdgpu_buffer_rsrc_t mk_slot_rsrc(int32_t *b)");
        e.line("{");
        e.line("    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)(256u * MK_HBM_NSLOTS), 0x00020000);");
        e.line("}");
        e.line("#define MK_SLOT_LANE ((int32_t)((threadIdx.x & 63u) * 4u))");
        e.line("MK_FN void mk_slot_st(int32_t *b, uint32_t s, int32_t v)");
        e.line("{");
        e.line("    if (s < MK_SLOTS_LDS_N) MK_LDS_SLOTS[MK_LDS_IX(s)] = v;");
        e.line("    else __builtin_amdgcn_raw_buffer_store_b32(v, mk_slot_rsrc(b), (int32_t)((uint32_t)MK_SLOT_LANE + (s - MK_SLOTS_LDS_N) * 256u), 0, 0);");
        e.line("}");
        e.line("MK_FN int32_t mk_slot_ld(int32_t *b, uint32_t s)");
        e.line("{");
        e.line("    if (s < MK_SLOTS_LDS_N) return MK_LDS_SLOTS[MK_LDS_IX(s)];");
        e.line("    return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(mk_slot_rsrc(b), (int32_t)((uint32_t)MK_SLOT_LANE + (s - MK_SLOTS_LDS_N) * 256u), 0, 0);");
        e.line("}");
        e.line("#undef MK_SLOT_ST");
        e.line("#undef MK_SLOT_LD");
        e.line("#undef MK_SLOT_STX");
        e.line("#undef MK_SLOT_LDX");
        e.line("#define MK_SLOT_ST(b, ss, s, v) mk_slot_st((b), (uint32_t)(s), (int32_t)(v))");
        e.line("#define MK_SLOT_LD(b, ss, s) mk_slot_ld((b), (uint32_t)(s))");
        e.line("#define MK_SLOT_STX(b, ss, s, v) MK_SLOT_ST(b, ss, s, v)");
        e.line("#define MK_SLOT_LDX(b, ss, s) MK_SLOT_LD(b, ss, s)");
        e.line("#endif");
    } else if (nl) {
        // Heavy kernel, slots in LDS: one wave per block owns nslots x 64
        // words, slot s of lane l at MK_LDS_IX(s) (a wave's access is 64
        // consecutive words, or 64 consecutive 16-byte quads: conflict-free).
        // No HBM traffic for the stacks.
        e.line("#ifndef MK_LANE_CHECKED");
        e.line("#define MK_SLOTS_LDS 1");
        e.line("__shared__ int32_t mk_lds_slots[MK_NSLOTS * 64u];");
        emit_lds_access(e, *g.lim);
        e.line("#define MK_SLOT_IX(s) MK_LDS_IX(s)");
        e.line("#undef MK_SLOT_ST");
        e.line("#undef MK_SLOT_LD");
        e.line("#undef MK_SLOT_STX");
        e.line("#undef MK_SLOT_LDX");
        e.line("#define MK_SLOT_ST(b, ss, s, v) (MK_LDS_SLOTS[MK_SLOT_IX(s)] = (int32_t)(v))");
        e.line("#define MK_SLOT_LD(b, ss, s) (MK_LDS_SLOTS[MK_SLOT_IX(s)])");
        e.line("#define MK_SLOT_STX(b, ss, s, v) MK_SLOT_ST(b, ss, s, v)");
        e.line("#define MK_SLOT_LDX(b, ss, s) MK_SLOT_LD(b, ss, s)");
        e.line("#endif");
    } else if (blocked && g.ndops > g.lim->heavy_ops) {
        // Heavy kernel, wave-blocked: `slots` is the wave's block (wave-uniform)
        // and a slot access is a buffer op whose slot offset s * 256 is a
        // scalar (SGPR + immediate) and whose lane offset is one VGPR, so no
        // 64-bit per-lane address is formed or kept live per slot (a deep
        // pipeline's straight-line pushes otherwise hoist dozens of them).
        e.line("#ifndef MK_LANE_CHECKED");
        e.line("#define MK_SLOTS_BUFFER 1");
        e.line("MK_FN __amdgpu_buffer_rsrc_t mk_slot_rsrc(int32_t *b)");
        e.line("{");
        e.line("    return __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)(256u * MK_NSLOTS), 0x00020000);");
        e.line("}");
        e.line("#define MK_SLOT_LANE ((int32_t)((threadIdx.x & 63u) * 4u))");
        e.line("#undef MK_SLOT_ST");
        e.line("#undef MK_SLOT_LD");
        e.line("#define MK_SLOT_ST(b, ss, s, v) \\");
        e.line("    __builtin_amdgcn_raw_buffer_store_b32((v), mk_slot_rsrc(b), MK_SLOT_LANE, (int32_t)((uint32_t)(s) * 256u), 0)");
        e.line("#define MK_SLOT_LD(b, ss, s) \\");
        e.line("    ((int32_t)__builtin_amdgcn_raw_buffer_load_b32(mk_slot_rsrc(b), MK_SLOT_LANE, (int32_t)((uint32_t)(s) * 256u), 0))");
        // a per-lane slot number goes into the vector offset
        e.line("#undef MK_SLOT_STX");
        e.line("#undef MK_SLOT_LDX");
        e.line("#define MK_SLOT_STX(b, ss, s, v) \\");
        e.line("    __builtin_amdgcn_raw_buffer_store_b32((v), mk_slot_rsrc(b), (int32_t)((uint32_t)MK_SLOT_LANE + (uint32_t)(s) * 256u), 0, 0)");
        e.line("#define MK_SLOT_LDX(b, ss, s) \\");
        e.line("    ((int32_t)__builtin_amdgcn_raw_buffer_load_b32(mk_slot_rsrc(b), (int32_t)((uint32_t)MK_SLOT_LANE + (uint32_t)(s) * 256u), 0, 0))");
        e.line("#endif");
    }
    if (checked) { // host tests only: the GPU kernel serves unguarded launches
        e.line("#ifdef MK_LANE_CHECKED");
        emit_stream_lane(p, g, e, "mk_lane", false);
        e.line("#endif");
    }
    emit_stream_lane(p, g, e, "mk_lane_ng", true);
}

// ---- machine shape: resumable lane --------------------------------------------

// A fast variant that loops on itself: GUARD, data micro-ops, then BR or JUMP
// with itself as a target (emit_self_loop).
bool self_loop(const Graph &g, uint32_t v, size_t &guard_pc, size_t &exit_pc)
{
    if (v & 1u) return false;
    size_t pc = g.entry[v];
    if (g.D[pc].op != U_GUARD) return false;
    guard_pc = pc++;
    for (;; ++pc) {
        const DOp &I = g.D[pc];
        switch (I.op) {
        case U_MOV: case U_LI: case U_ADD: case U_SUB: case U_ADDI: case U_RSUBI: case U_ST: case U_STI: case U_LD:
        case U_STX: case U_LDX: case U_OVF:
            continue;
        case U_BRX: // a side exit at the loop head (a dynamic POP's empty check) only
            if (pc != guard_pc + 1 || (uint32_t)I.imm == v) return false;
            continue;
        case U_JUMP:
            exit_pc = pc;
            return (uint32_t)I.imm == v;
        case U_BR:
            exit_pc = pc;
            return (uint32_t)(uint64_t)I.imm == v || (uint32_t)((uint64_t)I.imm >> 32) == v;
        default: return false;
        }
    }
}

// Self-loop v as a wave-uniform loop with per-lane predication.  The lanes
// of the group run the body together; a lane's flag `a` drops once it leaves
// the loop (branch not taken, or the next iteration's budget guard fails) and
// from then on its registers stay frozen (selects), so the loop control is
// scalar and no divergent branch or exec-mask bookkeeping is paid per
// iteration.  The wave checks every kLoopUnroll iterations whether enough of
// the group is still in the loop (MK_KEEP), so a few long trips do not hold
// the others.
//
// Two phases.  At entry the wave has the largest step count of its lanes
// (smax, from the dispatcher) and from it the number of iterations T that no lane's budget
// guard can stop; those run unguarded and without step counting -- a lane's
// steps are recovered at the end from its trip count, read off an induction
// register (a register the body only bumps by a constant, whose bump is
// predicated instead of selected) or, without one, a per-lane counter.  Only
// iterations past T (a launch whose budget ends inside the loop) run the
// guarded body, which keeps steps exact per iteration.
constexpr int kLoopUnroll = 4; // guarded phase
// Unguarded phases: iterations per exit test, by body size in micro-ops (a
// test costs ~13 SALU; C5's 1-op bodies on MI355X: 4 -> 578 us, 8 -> 426,
// 16 -> 401, 32 -> 391).
int fast_unroll(size_t body_ops) { return body_ops <= 2 ? 32 : body_ops <= 4 ? 16 : body_ops <= 8 ? 8 : 4; }

enum LoopMode { LOOP_GUARDED, LOOP_WIDE, LOOP_NARROW };

// Narrow phase of a loop whose body is only the induction bump x += imm and
// whose stay condition tests x: the flag can be an int 0/1 from one
// full-rate VALU op (MK_FLAG_*: x > 0 by med3(x, 0, 1), x < 0 by x >> 31,
// x != 0 by min_u32(x, 1)) instead of a lane mask.  Returns the macro, or
// null when the loop does not have that form.
const char *int_flag_fn(const DOp &X, uint32_t v, int ind, size_t body_ops, int64_t step)
{
    if (X.op != U_BR || (int)(X.a / 8) != ind || body_ops != 1) return nullptr;
    if (!(step == 1 || step == -1 || (step > -(1 << 23) && step < (1 << 23)))) return nullptr;
    const uint32_t tk = (uint32_t)(uint64_t)X.imm, nt = (uint32_t)((uint64_t)X.imm >> 32);
    if (tk == nt) return nullptr;
    const bool neg = tk != v; // the loop continues when the condition fails
    switch ((X.fl >> UF_COND_SHIFT) & 3u) {
    case 0: return neg ? "MK_FLAG_NZ" : nullptr; // stay while x != 0 (JEZ leaves)
    case 1: return neg ? nullptr : "MK_FLAG_NZ";
    case 2: return neg ? nullptr : "MK_FLAG_GT";
    case 3: return neg ? nullptr : "MK_FLAG_LT";
    }
    return nullptr;
}

void emit_self_loop(const OpWriter &w, const Graph &g, uint32_t v, size_t gpc, size_t xpc)
{
    Emitter &e = w.e;
    const DOp &G = g.D[gpc], &X = g.D[xpc];
    // registers the body reads or writes, the ones it writes, and how often
    const size_t nr = g.used_reg.size();
    std::vector<char> rd(nr, 0), wr(nr, 0);
    std::vector<int> nwr(nr, 0);
    auto R = [&](uint32_t off) { rd[off / 8] = 1; };
    auto W = [&](uint32_t off) { wr[off / 8] = rd[off / 8] = 1; ++nwr[off / 8]; };
    for (size_t pc = gpc + 1; pc < xpc; ++pc) {
        const DOp &I = g.D[pc];
        switch (I.op) {
        case U_MOV: case U_ADDI: case U_RSUBI: R(I.a); W(I.d); break;
        case U_ADD: case U_SUB: R(I.a); R(I.b); W(I.d); break;
        case U_LI: case U_LD: W(I.d); break;
        case U_ST: R(I.a); break;
        case U_STX: R(I.a); R(I.b); break;
        case U_LDX: R(I.b); W(I.d); break;
        case U_OVF: R(I.b); if (I.fl & UF_OUTREG) R(I.a); break;
        case U_BRX: R(I.a); break;
        default: break;
        }
    }
    // A PUSH onto a dynamic stack in the body (OVF): a lane at the capacity
    // leaves the loop there -- its flag drops, the iteration's register writes
    // are discarded by the selects and its steps stop at the iteration's
    // start; the OVF's step count, status and output are recorded and applied
    // after the loop.  Trip counts then come from the per-lane counter.
    // A BRX at the head (a dynamic POP's empty check, before any other op)
    // leaves likewise: the lane's registers are the iteration's start, its
    // step count the loop's so far, and it continues at the BRX's target.
    bool ovf = false;
    for (size_t pc = gpc + 1; pc < xpc; ++pc) ovf = ovf || g.D[pc].op == U_OVF || g.D[pc].op == U_BRX;
    const DOp *brx = g.D[gpc + 1].op == U_BRX ? &g.D[gpc + 1] : nullptr;
    // induction register: written once per iteration, by r += imm (no
    // truncation).  Loops with an OVF / BRX exit have one too since round 6
    // (a dynamic PUSH loop's depth register): the exit drops the lane's flag
    // before the bump, so the bumps count exactly the iterations completed,
    // as the per-lane counter did; the register then needs no select and
    // runs in 32 bits in the narrow phase (t2_dyn_depth 130 -> ? us).
    int ind = -1;
    int64_t step = 0;
    for (size_t pc = gpc + 1; pc < xpc && ind < 0; ++pc) {
        const DOp &I = g.D[pc];
        if (I.op == U_ADDI && I.a == I.d && !(I.fl & UF_TA) && nwr[I.d / 8] == 1 && I.imm != 0 &&
            I.imm > -(int64_t(1) << 31) && I.imm < (int64_t(1) << 31))
            ind = (int)(I.d / 8), step = I.imm;
    }
    std::string c = "true";
    uint32_t other = v;
    // In the unguarded phases a lane that left keeps its registers, so the
    // exit condition on a register that only changes when the lane is active
    // (the induction register, or one the body never writes) stays false:
    // there `a` is the condition itself, one compare and no mask AND.
    const bool cond_is_flag = !ovf && X.op == U_BR && ((int)(X.a / 8) == ind || !wr[X.a / 8]);
    if (X.op == U_BR) {
        R(X.a);
        const uint32_t tk = (uint32_t)(uint64_t)X.imm, nt = (uint32_t)((uint64_t)X.imm >> 32);
        OpWriter n{e, w.p, "n"};
        if (tk == v && nt != v) c = n.cond(X), other = nt;
        else if (tk != v) c = "!" + n.cond(X), other = tk;
    }
    // One iteration.  GUARDED: steps counted and the budget checked per
    // iteration.  WIDE: no guard, no step counting.  NARROW: as WIDE with the
    // induction register held in 32 bits (x; exact while it stays in range).
    auto iteration = [&](LoopMode mode) {
        e.line("    {");
        for (uint32_t r = 0; r < nr; ++r) {
            if (!rd[r]) continue;
            if (mode == LOOP_NARROW && (int)r == ind) e.line("    int64_t n%u = (int64_t)x;", r);
            else e.line("    int64_t n%u = L.r%u;", r, r);
        }
        OpWriter n{e, w.p, "n"};
        for (size_t pc = gpc + 1; pc < xpc; ++pc) {
            const DOp &I = g.D[pc];
            // stores, and indexed loads (a lane that left may hold any index), only for lanes in the loop
            if (I.op == U_ST || I.op == U_STI || I.op == U_STX || I.op == U_LDX) e.line("    if (a)");
            if (I.op == U_BRX) {
                e.line("    {");
                e.line("    const bool x_ = a && %s;", n.cond(I).c_str());
                e.line("    brx_ = brx_ || x_;");
                e.line("    a = a && !x_;");
                e.line("    }");
            } else if (I.op == U_OVF) {
                e.line("    {");
                e.line("    const bool o_ = a && %s;", n.ovf_cond(I).c_str());
                e.line("    if (o_) { ovf_ = true; ovs_ = %uu; ovst_ = %uu; ovo_ = %s; }", I.inc, I.d, n.ovf_result(I).c_str());
                e.line("    a = a && !o_;");
                e.line("    }");
            } else if (I.op == U_ADDI && (int)(I.d / 8) == ind) {
                if (mode == LOOP_NARROW) {
                    if (I.imm == 1 || I.imm == -1) // x -/+ a: one subtract/add with the mask as carry
                        e.line("    x = (int32_t)((uint32_t)x %c (uint32_t)a);", I.imm < 0 ? '-' : '+');
                    else
                        e.line("    x = (int32_t)((uint32_t)x + (a ? %uu : 0u));", (uint32_t)(int32_t)I.imm);
                    e.line("    n%d = (int64_t)x;", ind);
                } else {
                    e.line("    n%d = (int64_t)((uint64_t)n%d + (a ? %s : 0ull));", ind, ind, u64lit(I.imm).c_str());
                }
            } else {
                n.data(I);
            }
        }
        for (uint32_t r = 0; r < nr; ++r) {
            if (!wr[r]) continue;
            if ((int)r == ind) {
                if (mode != LOOP_NARROW) e.line("    L.r%u = n%u;", r, r);
            } else {
                e.line("    L.r%u = a ? n%u : L.r%u;", r, r, r);
            }
        }
        if (mode == LOOP_GUARDED) {
            e.line("    L.steps += a ? %uu : 0u;", X.inc);
            e.line("    a = a & (%s) & (L.steps < lim);", c.c_str());
        } else {
            if (ind < 0) e.line("    k += a ? 1u : 0u;");
            if (cond_is_flag) e.line("    a = %s;", c.c_str());
            else e.line("    a = a & (%s);", c.c_str());
        }
        e.line("    }");
    };
    int uf = fast_unroll(xpc - gpc - 1);
    if (g.lim->loop_unroll >= 1 && g.lim->loop_unroll <= 64) uf = g.lim->loop_unroll; // MK_JIT_LOOP_UNROLL
    // Saturating countdowns (counter c >= 0 per lane, 0 once it left): chunks
    // of 2 uf decrements while some lane still needs more than uf, then the
    // uf chunks -- half the exit tests on long trips, and no more idle
    // iterations than uf chunks alone (a 2 uf chunk starts only when a lane
    // needs over uf of them).  MK_JIT_SAT_TIER=0: uf chunks only.
    auto emit_sat_tier = [&](const char *c) {
        e.line("    while (more && T32 - it >= %uu && MK_KEEP(%s > %d, need)) {", 2 * uf, c, uf);
        e.line("    it += %uu;", 2 * uf);
        if (uf % (int)g.lim->sat_block == 0)
            for (int u = 0; u < 2 * uf; u += (int)g.lim->sat_block) e.line("    %s = MK_SATDECB(%s);", c, c);
        else
            for (int u = 0; u < 2 * uf; ++u) e.line("    %s = MK_SATDEC(%s);", c, c);
        e.line("    }");
        e.line("    more = MK_KEEP(%s != 0, need);", c);
    };
    // an unguarded phase: chunks of uf iterations while T allows
    auto phase = [&](LoopMode mode, const char *cap) {
        e.line("    while (more && %s - it >= %uu) {", cap, uf);
        e.line("    it += %uu;", uf);
        for (int u = 0; u < uf; ++u) iteration(mode);
        e.line("    more = MK_KEEP(a, need);");
        e.line("    }");
    };
    // guard: steps + g >= budget  <=>  steps >= lim (lim = 0 when budget <= g)
    e.line("    const uint32_t lim = budget > %uu ? budget - %uu : 0u;", G.inc, G.inc);
    e.line("    if (L.steps >= lim) {");
    e.line("        L.sb = %uu;", (uint32_t)G.imm);
    e.line("        break;");
    e.line("    }");
    e.line("    const uint32_t need = MK_LOOP_NEED(pol);");
    e.line("    MK_PRIO_LOOP();");
    e.line("    bool a = true, more = true;");
    if (ovf) {
        e.line("    bool ovf_ = false, brx_ = false;");
        e.line("    uint32_t ovs_ = 0u, ovst_ = 0u;");
        e.line("    int32_t ovo_ = 0;");
        e.line("    (void)brx_; (void)ovs_; (void)ovst_; (void)ovo_;");
    }
    e.line("    {");
    e.line("    const uint32_t s0 = L.steps;");
    if (ind >= 0) e.line("    const int64_t i0 = L.r%d;", ind);
    else e.line("    uint32_t k = 0u;");
    // after j iterations a lane has steps <= smax + j*inc (smax is uniform, so
    // is T; it may count lanes of the group that stopped at the guard above:
    // then T = 0)
    e.line("    const uint32_t T = smax < lim ? (lim - 1u - smax) / %uu : 0u;", X.inc);
    e.line("    uint32_t it = 0u;");
    if (ind >= 0) {
        // |x| <= 2^30 at entry and at most (2^30 - 1) / |imm| iterations: x stays in int32
        const uint64_t ad = step < 0 ? (uint64_t)(-step) : (uint64_t)step;
        e.line("    if (T >= %uu && MK_ALL(L.r%d >= -0x40000000ll && L.r%d <= 0x40000000ll)) {", uf, ind, ind);
        e.line("    const uint32_t T32 = T < %lluu ? T : %lluu;", (unsigned long long)(0x3fffffffull / ad),
               (unsigned long long)(0x3fffffffull / ad));
        e.line("    int32_t x = (int32_t)L.r%d;", ind);
        if (const char *flag = int_flag_fn(X, v, ind, xpc - gpc - 1, step)) {
            // the whole body is the induction bump: the flag as an int 0/1,
            // no lane masks (mask-writing VALU ops issue at half rate)
            e.line("    int32_t f = 1;");
            // A countdown by 1 (x > 0, x -= 1): past its first iteration a
            // lane still in the loop has x > 0 (sat, below).
            const bool gt = !std::strcmp(flag, "MK_FLAG_GT"), lt = !std::strcmp(flag, "MK_FLAG_LT");
            const bool sat = step == -1 && gt;
            if (!sat && g.lim->sat_count && ((gt && step <= -2) || (lt && step >= 1))) {
                // Counter form (MK_JIT_SAT_COUNT, round 4): a countdown by k
                // (x > 0, x -= k; or x < 0, x += k) from x1 after the first
                // iteration runs z = ceil(|x1| / k) more iterations, so each
                // iteration is one saturating decrement of z (v_sub_u32
                // clamp: full rate on gfx950) instead of the bump and the
                // flag (v_mad_i32_i24 + v_med3_i32: half rate each,
                // tools/probe/valu_rates.hip); x follows from the iterations
                // run, exactly, at the loop's end -- also when the budget
                // bound T32 stops it first.
                const uint64_t k = (uint64_t)(step < 0 ? -step : step);
                e.line("    it = 1u;");
                e.line("    x = (int32_t)((uint32_t)x + %uu);", (uint32_t)(int32_t)step);
                e.line("    (void)f;");
                e.line("    const int32_t f0 = %s(x);", flag);
                e.line("    const uint32_t z0 = f0 ? ((uint32_t)(%sx) + %lluu) / %lluu : 0u;", gt ? "" : "-",
                       (unsigned long long)(k - 1), (unsigned long long)k);
                e.line("    int32_t z = (int32_t)z0;");
                e.line("    more = MK_KEEP(z != 0, need);");
                emit_sat_tier("z");
                e.line("    while (more && T32 - it >= %uu) {", uf);
                e.line("    it += %uu;", uf);
                if (uf % (int)g.lim->sat_block == 0) // sat_block decrements per asm block
                    for (int u = 0; u < uf; u += (int)g.lim->sat_block) e.line("    z = MK_SATDECB(z);");
                else
                    for (int u = 0; u < uf; ++u) e.line("    z = MK_SATDEC(z);");
                e.line("    more = MK_KEEP(z != 0, need);");
                e.line("    }");
                e.line("    a = z != 0;");
                e.line("    x = (int32_t)((uint32_t)x + %uu * (z0 - (uint32_t)z));", (uint32_t)(int32_t)step);
            } else if (sat) {
                // Past the first iteration a lane still in the loop has x > 0:
                // one saturating decrement per iteration (v_sub_u32 clamp), a
                // lane that left holds 0 and its flag is x != 0.  Lanes that
                // left at the first test are parked at 0 and get their x back.
                e.line("    it = 1u;");
                e.line("    x = (int32_t)((uint32_t)x - 1u);");
                e.line("    (void)f;");
                e.line("    const int32_t f0 = MK_FLAG_GT(x), x0 = x;");
                e.line("    x = f0 ? x : 0;");
                e.line("    more = MK_KEEP(x != 0, need);");
                emit_sat_tier("x");
                e.line("    while (more && T32 - it >= %uu) {", uf);
                e.line("    it += %uu;", uf);
                if (uf % (int)g.lim->sat_block == 0)
                    for (int u = 0; u < uf; u += (int)g.lim->sat_block) e.line("    x = MK_SATDECB(x);");
                else
                    for (int u = 0; u < uf; ++u) e.line("    x = MK_SATDEC(x);");
                e.line("    more = MK_KEEP(x != 0, need);");
                e.line("    }");
                e.line("    a = x != 0;");
                e.line("    x = f0 ? x : x0;");
            } else {
                e.line("    while (more && T32 - it >= %uu) {", uf);
                e.line("    it += %uu;", uf);
                for (int u = 0; u < uf; ++u) {
                    if (step == 1 || step == -1)
                        e.line("    x = (int32_t)((uint32_t)x %c (uint32_t)f);", step < 0 ? '-' : '+');
                    else
                        e.line("    x = MK_MAD24(f, %d, x);", (int)step);
                    e.line("    f = %s(x);", flag);
                }
                e.line("    more = MK_KEEP(f != 0, need);");
                e.line("    }");
                e.line("    a = f != 0;");
            }
        } else {
            phase(LOOP_NARROW, "T32");
        }
        e.line("    L.r%d = (int64_t)x;", ind);
        e.line("    }");
    }
    phase(LOOP_WIDE, "T");
    if (ind >= 0) {
        // iterations = (r - i0) / step, an exact quotient below 2^32 (steps
        // are 32-bit): |r - i0| >> ctz(step) times the inverse of step's odd
        // part mod 2^32 -- one 32-bit multiply instead of a signed 64-bit
        // division (round 6)
        const uint64_t ad = step < 0 ? (uint64_t)(-step) : (uint64_t)step;
        const int sh = __builtin_ctzll(ad);
        const uint32_t odd = (uint32_t)(ad >> sh);
        uint32_t inv = odd; // Newton: each step doubles the correct low bits (3 -> 6 -> 12 -> 24 -> 48)
        for (int k = 0; k < 4; ++k) inv *= 2u - odd * inv;
        const char *y = step < 0 ? "((uint64_t)i0 - (uint64_t)L.r%d)" : "((uint64_t)L.r%d - (uint64_t)i0)";
        std::string ys(64, '\0');
        ys.resize((size_t)std::snprintf(&ys[0], ys.size(), y, ind));
        if (odd == 1u)
            e.line("    L.steps = s0 + %uu * (uint32_t)(%s >> %d);", X.inc, ys.c_str(), sh);
        else
            e.line("    L.steps = s0 + %uu * ((uint32_t)(%s >> %d) * %uu);", X.inc, ys.c_str(), sh, inv);
    } else
        e.line("    L.steps = s0 + %uu * k;", X.inc);
    e.line("    }");
    e.line("    if (more) {");
    e.line("    do {");
    for (int u = 0; u < kLoopUnroll; ++u) iteration(LOOP_GUARDED);
    e.line("    } while (MK_KEEP(a, need));");
    e.line("    }");
    e.line("    MK_PRIO_REST();");
    // a: still in the loop (suspended); otherwise it left through the branch
    // (the condition on its frozen registers fails) or through the guard
    if (brx) {
        e.line("    if (brx_) {");
        e.line("        L.steps += %uu;", brx->inc);
        e.line("        L.sb = %uu;", (uint32_t)brx->imm);
        e.line("        break;");
        e.line("    }");
    }
    if (ovf) {
        e.line("    if (ovf_) {");
        e.line("        L.steps += ovs_;");
        e.line("        L.st = ovst_;");
        e.line("        L.outv = ovo_;");
        e.line("        L.sb = MK_SB_DONE;");
        e.line("        break;");
        e.line("    }");
    }
    OpWriter l{e, w.p, "L.r"};
    std::string cl = "true";
    if (X.op == U_BR) {
        const uint32_t tk = (uint32_t)(uint64_t)X.imm, nt = (uint32_t)((uint64_t)X.imm >> 32);
        if (tk == v && nt != v) cl = l.cond(X);
        else if (tk != v) cl = "!" + l.cond(X);
    }
    e.line("    L.sb = (a || (%s)) ? (L.steps < lim ? %uu : %uu) : %uu;", cl.c_str(), v, (uint32_t)G.imm, other);
    e.line("    break;");
    e.line("    }");
}

void emit_machine_lane(const SchedProgram &p, const Graph &g, Emitter &e)
{
    OpWriter w{e, p, "L.r"};
    const size_t nv = g.entry.size();
    std::vector<uint32_t> loops;
    e.line("// generated from a compiled schedule: %zu variants reachable, %zu micro-ops, cyclic", g.nreach, g.ndops);
    e.line("#define MK_JIT_MACHINE 1");
    { // wave priority around self-loops (the module header); none in host builds
        e.line("#ifndef MK_PRIO_LOOP");
        e.line("#define MK_PRIO_LOOP()");
        e.line("#define MK_PRIO_REST()");
        e.line("#endif");
    }
    { // host builds: sat_block plain decrements (the device prelude's asm block wins)
        e.line("#ifndef MK_SATDECB");
        e.line("#define MK_SATDECB(x) ([](int32_t v_) { for (int k_ = 0; k_ < %u; ++k_) v_ = MK_SATDEC(v_); return v_; }(x))",
               g.lim->sat_block);
        e.line("#endif");
    }
    e.line("#ifndef MK_CTABLE");
    e.line("#define MK_CTABLE static const");
    e.line("#endif");
    e.line("#define MK_SB_DONE 0xFFFFFFFEu");
    e.line("#define MK_SB_IDLE 0xFFFFFFFFu");
    if (p.session) {
        e.line("#define MK_SS_HANDOFF 0xFEu");     // L.st of a lane handed to the interpreter
        e.line("#define MK_SS_DEAD 0xFFFFFFF0u");  // session ended (stack overflow)
        e.line("#define MK_SS_T1 0xFFFFFFF1u");    // the interpreter holds the session
        e.line("#define MK_SS_HAND 0xFFFFFFF2u");  // handed off in this launch (the interpreter kernel imports it, sess_import_one)
    }
    {
        uint32_t used = 0;
        for (uint32_t r = 0; r < p.nregs; ++r) used += g.used_reg[r] ? 1u : 0u;
        e.line("#define MK_LANE_REGS %uu", used); // 64-bit lane registers (kMachineSortKernel's occupancy)
        // kMachineSortKernel's tile (JitLimits::ts_rounds = 0): 8 rounds of
        // 256 lanes when the lane has no stack slots (C5 211 vs 215 us), 4
        // with them (the census classes' slots in flight, r02v)
        e.line("#ifndef MK_TS_R");
        e.line("#define MK_TS_R %uu", p.nslots ? 4u : 8u);
        e.line("#endif");
    }
    e.line("struct MkLane {");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    int64_t r%u;", r);
    e.line("    uint32_t sb, steps, st;");
    e.line("    int32_t outv;");
    if (p.session) e.line("    uint32_t next; // sessions: where the next call starts (MK_SS_* markers)");
    e.line("};");
    if (p.session) {
        // the persistent lane state of a session between calls (mk_sess_exec):
        // its registers, [register][session] in HBM
        e.line("MK_FN void mk_sess_input(MkLane &L, int64_t x) { L.r%u = x; }", p.in_reg);
        e.line("MK_FN void mk_sess_load(MkLane &L, const int64_t *regs, uint64_t i, uint64_t n, bool on)");
        e.line("{");
        for (uint32_t r = 0; r < p.nregs; ++r)
            if (g.used_reg[r]) e.line("    L.r%u = on ? regs[%lluull * n + i] : 0;", r, (unsigned long long)r);
        e.line("}");
        e.line("MK_FN void mk_sess_store(const MkLane &L, int64_t *regs, uint64_t i, uint64_t n)");
        e.line("{");
        for (uint32_t r = 0; r < p.nregs; ++r)
            if (g.used_reg[r]) e.line("    regs[%lluull * n + i] = L.r%u;", (unsigned long long)r, r);
        e.line("}");
    }
    e.line("MK_FN void mk_init(MkLane &L, int64_t in)");
    e.line("{");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    L.r%u = 0;", r);
    e.line("    L.r%u = (int64_t)(int32_t)in;", p.in_reg);
    e.line("    L.sb = 0u;");
    e.line("    L.steps = 0u;");
    e.line("    L.st = 0u;");
    e.line("    L.outv = 0;");
    e.line("}");
    // The pool kernel's parked lanes (kMachinePoolKernel): a lane between
    // superblocks is its registers, superblock and step count (out / status
    // are set only on the way to MK_SB_DONE, when the lane is retired, never
    // parked), plus the input index it answers.  Struct of arrays in LDS.
    e.line("#define MK_NV %zuu", nv);
    e.line("#ifdef MK_POOL");
    e.line("struct MkPool {");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    int64_t r%u[MK_POOL];", r);
    e.line("    uint64_t idx[MK_POOL];");
    e.line("    uint32_t sb[MK_POOL];");
    e.line("    uint32_t steps[MK_POOL];");
    e.line("};");
    e.line("MK_FN void mk_park(MkPool &P, const uint32_t s, const MkLane &L, const uint64_t idx)");
    e.line("{");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    P.r%u[s] = L.r%u;", r, r);
    e.line("    P.idx[s] = idx;");
    e.line("    P.steps[s] = L.steps;");
    e.line("    P.sb[s] = L.sb;");
    e.line("}");
    e.line("MK_FN void mk_unpark(const MkPool &P, const uint32_t s, MkLane &L, uint64_t &idx)");
    e.line("{");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (g.used_reg[r]) e.line("    L.r%u = P.r%u[s];", r, r);
    e.line("    idx = P.idx[s];");
    e.line("    L.steps = P.steps[s];");
    e.line("    L.sb = P.sb[s];");
    e.line("    L.st = 0u;");
    e.line("    L.outv = 0;");
    e.line("}");
    e.line("#endif");
    // mk_run(u, ...): superblock variant u for a lane sitting on it (L.sb == u).
    // MK_LOOP_NEED() / MK_KEEP(m, need) come from the includer: the wave's
    // policy for leaving a loop early so that finished lanes can refill.
    // smax: at least the steps of every lane of the group (self-loops size
    // their unguarded phase from it; the kernel reduces it over the wave for
    // loop variants only, see mk_is_loop).
    Emitter tab; // budget-exit tables of checked variants (before mk_run)
    // The kernels call mk_run(u, L) under `if (L.sb == u)`; GVN then
    // replaces u by the lane's L.sb inside the branch and lowers the switch
    // as a divergent one: a compare-and-mask tree, one level per halving of
    // the variants.  The kernels pass MK_SCALAR(u), computed before the
    // branch; as mk_scalar (the module header: an empty asm with an SGPR
    // result, no instruction, that GVN cannot see through) the switch is a
    // scalar compare tree, but LLVM then copies the lane registers into and
    // out of every case.  Measured (r04u, bench launch times, scalar vs
    // divergent): C5 (36 variants) 123.7 vs 142.7 us, two_stacks (26) 237.8
    // vs 228.4, dyn_depth (15) 134.6 vs 134.6, jro_heavy (6) 59.0 vs 52.4 ms;
    // so the scalar switch from 32 reachable variants (MK_JIT_UNIFORM_SW=1|0
    // forces either).
    {
        const bool scalar = g.nreach >= 32;
        e.line(scalar ? "#define MK_SCALAR(u) mk_scalar(u)" : "#define MK_SCALAR(u) (u)");
    }
    const size_t fn_start = e.s.size();
    e.line("MK_FN void mk_run(const uint32_t u, MkLane &L, const uint32_t budget, int32_t *__restrict__ slots,");
    e.line("                  const uint64_t sstride, const uint32_t pol, const uint32_t smax)");
    e.line("{");
    // Variant v's code (guard, body, exit op) up to the label `lab:`, its
    // early exits jumping there.
    auto emit_plain = [&](uint32_t v, const std::string &lab) {
        const DOp &G = g.D[g.entry[v]];
        if (G.op == U_GUARD) {
            e.line("    if ((uint64_t)L.steps + %uu >= (uint64_t)budget) {", G.inc);
            e.line("        L.sb = %uu;", (uint32_t)G.imm);
            e.line("        goto %s;", lab.c_str());
            e.line("    }");
        }
        size_t lo, hi;
        body_range(g, v, lo, hi);
        const std::string fin = "L.sb = MK_SB_DONE; goto " + lab + ";", go = "L.sb = %uu; goto " + lab + ";";
        emit_body(w, g, v, lo, hi, [&](const DOp &I, const char *inc, size_t) {
            emit_inline_end(w, I, inc, "L.", fin.c_str(), go.c_str());
        });
        const DOp &I = g.D[hi];
        switch (I.op) {
        case U_JUMP:
            e.line("    L.steps += %uu;", I.inc);
            e.line("    L.sb = %uu;", (uint32_t)I.imm);
            break;
        case U_BR:
            e.line("    L.steps += %uu;", I.inc);
            e.line("    L.sb = %s ? %uu : %uu;", w.cond(I).c_str(), (uint32_t)(uint64_t)I.imm,
                   (uint32_t)((uint64_t)I.imm >> 32));
            break;
        case U_JRO: {
            e.line("    L.steps += %uu;", I.inc);
            e.line("    {");
            w.jro_target(I);
            // The successor table packed into at most four 64-bit constants
            // (W-bit entries, 64 / W per word): a select of the word and a
            // shift (round 6).  The select chain below it LLVM turns into a
            // switch, which a divergent t lowers as a tree of exec-masked
            // branches: ~120 instructions for C5's 15 arms.
            uint32_t top = 0;
            for (uint32_t t = 0; t <= I.b; ++t) top = std::max(top, p.jtab[(size_t)I.imm + t]);
            const uint32_t W = top < 16u ? 4u : top < 256u ? 8u : 16u, P = 64u / W;
            const uint32_t words = (I.b + 1u + P - 1u) / P;
            if (top < 65536u && words <= 4u) {
                std::string sel;
                for (uint32_t k = 0; k < words; ++k) {
                    uint64_t word = 0;
                    for (uint32_t t = k * P; t < (k + 1u) * P && t <= I.b; ++t)
                        word |= (uint64_t)p.jtab[(size_t)I.imm + t] << (W * (t - k * P));
                    char b[96];
                    if (k + 1u < words) snprintf(b, sizeof b, "ti < %uu ? 0x%016llxull : ", (k + 1u) * P, (unsigned long long)word);
                    else snprintf(b, sizeof b, "0x%016llxull", (unsigned long long)word);
                    sel += b;
                }
                e.line("        const uint32_t ti = (uint32_t)t;");
                e.line("        const uint64_t tw = %s;", sel.c_str());
                e.line("        L.sb = (uint32_t)(tw >> (%uu * (ti & %uu))) & 0x%xu;", W, P - 1u, (1u << W) - 1u);
            } else {
                const uint32_t last = p.jtab[(size_t)I.imm + I.b];
                std::string sel;
                for (uint32_t t = 0; t < I.b; ++t) {
                    const uint32_t tgt = p.jtab[(size_t)I.imm + t];
                    if (tgt == last) continue;
                    char b[64];
                    snprintf(b, sizeof b, "t == %u ? %uu : ", t, tgt);
                    sel += b;
                }
                e.line("        L.sb = %s%uu;", sel.c_str(), last);
            }
            e.line("    }");
            break;
        }
        case U_END:
            e.line("    L.steps += %uu;", I.inc);
            e.line("    L.outv = %s;", w.result(I).c_str());
            e.line("    L.st = %uu;", I.d);
            e.line("    L.sb = MK_SB_DONE;");
            break;
        case U_YIELD: { // sessions: the call ends; the next starts at lo32(imm)
            char o[64];
            snprintf(o, sizeof o, "(int32_t)%" PRId32, (int32_t)((uint64_t)I.imm >> 32));
            e.line("    L.steps += %uu;", I.inc);
            e.line("    L.outv = %s;", (I.d & MK_ST_HAS_OUTPUT) ? ((I.fl & UF_OUTREG) ? w.result(I).c_str() : o) : "0");
            e.line("    L.st = %uu;", I.d);
            e.line("    L.next = %uu;", (uint32_t)(uint64_t)I.imm);
            e.line("    L.sb = MK_SB_DONE;");
            break;
        }
        case U_HANDOFF: // sessions: the interpreter finishes the call from this superblock's entry
            e.line("    L.st = MK_SS_HANDOFF;");
            e.line("    L.next = %uu;", (uint32_t)I.imm);
            e.line("    L.sb = MK_SB_DONE;");
            break;
        default: break;
        }
        e.line("    %s:", lab.c_str());
    };
    e.line("    (void)slots; (void)sstride; (void)budget; (void)pol; (void)smax;");
    e.line("    switch (u) {");
    for (uint32_t v = 0; v < nv; ++v) {
        if (!g.seen[v]) continue;
        e.line("    case %uu: {", v);
        size_t gpc = 0, xpc = 0;
        if (self_loop(g, v, gpc, xpc)) {
            loops.push_back(v);
            emit_self_loop(w, g, v, gpc, xpc);
            continue;
        }
        size_t lo, hi;
        body_range(g, v, lo, hi);
        const RoundEnds re = round_ends(g, v, lo, hi);
        if (!re.segs.empty() && !has_inline_exit(g, lo, hi)) { // checked variant: always ends at a round end (emit_budget_exit)
            const DOp &G = g.D[g.entry[v]];
            if (G.op == U_GUARD) {
                e.line("    if ((uint64_t)L.steps + %uu >= (uint64_t)budget) {", G.inc);
                e.line("        L.sb = %uu;", (uint32_t)G.imm);
                e.line("        goto X%u;", v);
                e.line("    }");
            }
            e.line("    int32_t mk_o = 0;");
            emit_body(w, g, v, lo, hi, [&](const DOp &I, const char *, size_t pc) {
                if (pc == re.snap_pc) e.line("    mk_o = %s;", w.result(I).c_str());
            });
            emit_budget_exit(e, tab, re, v, "L.steps");
            e.line("    L.steps += inc_;");
            e.line("    L.st = st_;");
            e.line("    L.outv = (st_ & %uu) ? mk_o : 0;", (unsigned)MK_ST_HAS_OUTPUT);
            e.line("    L.sb = MK_SB_DONE;");
            e.line("    (void)mk_o;");
            e.line("    X%u:", v);
            e.line("    break;");
            e.line("    }");
            continue;
        }
        emit_plain(v, "X" + std::to_string(v));
        e.line("    break;");
        e.line("    }");
    }
    e.line("    default: L.sb = MK_SB_DONE; break;");
    e.line("    }");
    e.line("}");
    e.s.insert(fn_start, tab.s);
    e.line("// %zu self-loops", loops.size());
    // the sweep dispatcher's order (JitLimits::sweep, kMachineSortKernel):
    // one pass over the variants in forward order runs every lane as far as
    // the graph's forward edges take it.  Machines of few variants keep the
    // rounds: their compare tree is shallow and a round cheap (jro_heavy, 6
    // variants: 52.3 ms by rounds, 58.8 by sweeps; C5, 36: 105.8 -> 97.0 us;
    // two_stacks and dyn_depth unchanged, profiles/r06w_sweep_census_ab.txt).
    // The kernel runs MK_SWEEP_PASSES passes, then rounds for the lanes left
    // (loops over several variants: each iteration would cost a whole pass),
    // and machines of very many variants keep the rounds (a 190-variant test
    // network: 220 ms by rounds, 403 ms with one pass first, 1,348 ms by
    // sweeps alone; profiles/r07l_sweep_random_ab.txt)
    if (g.lim->sweep && g.nreach >= kSweepMinVariants && g.nreach <= kSweepMaxVariants) {
        const std::vector<uint32_t> fo = forward_order(g);
        // the checked variants (a budget's last round: rare) go last, behind
        // one ballot over a mask of their ids, when the ids fit one (C5: 18
        // ballots per pass fewer, 95.4 -> 87.9 us, profiles/r07b_sweep_cold_ab.txt)
        auto checked = [&](uint32_t v) {
            size_t gpc = 0, xpc = 0, lo = 0, hi = 0;
            if (self_loop(g, v, gpc, xpc)) return false;
            body_range(g, v, lo, hi);
            return !round_ends(g, v, lo, hi).segs.empty() && !has_inline_exit(g, lo, hi);
        };
        bool split = true;
        for (uint32_t v : fo) split = split && (!checked(v) || v < 64u);
        std::string l = "#define MK_SWEEP_LIST(X)", c = "#define MK_SWEEP_COLD(X)";
        uint64_t mask = 0;
        for (uint32_t v : fo) {
            size_t gpc = 0, xpc = 0;
            const std::string x = " X(" + std::to_string(v) + "u, " + (self_loop(g, v, gpc, xpc) ? "1" : "0") + ")";
            if (split && checked(v)) c += x, mask |= 1ull << v;
            else l += x;
        }
        e.s += l + "\n";
        if (mask) {
            e.s += c + "\n";
            e.line("#define MK_SWEEP_COLD_MASK 0x%016" PRIx64 "ull", mask);
        }
    }
    e.line("MK_FN bool mk_is_loop(const uint32_t u)");
    e.line("{");
    if (loops.empty()) {
        e.line("    (void)u;");
        e.line("    return false;");
    } else {
        e.line("    switch (u) {");
        for (uint32_t v : loops) e.line("    case %uu:", v);
        e.line("        return true;");
        e.line("    default: return false;");
        e.line("    }");
    }
    e.line("}");
    if (p.session) return; // sessions: mk_sess_exec drives mk_run; no single-lane form
    // two lanes per thread in the tile-sorted kernel (MK_JIT_PAIR): one
    // sweep pass for two chunks; two lanes would share the thread's slot
    // column, and the phase profile (MK_JIT_PROF) times the one-lane form
    if (g.lim->pair && !p.nslots && g.lim->ts_rounds % 2u == 0u && !g.lim->prof) e.line("#define MK_PAIR 1");
    // the whole lane, for the CPU tests (the kernel drives mk_run itself)
    e.line("MK_FN int32_t mk_lane(int64_t in, uint32_t budget, int32_t *__restrict__ slots, uint64_t sstride,");
    e.line("                      uint32_t *steps_out, uint32_t *status_out)");
    e.line("{");
    e.line("    MkLane L;");
    e.line("    mk_init(L, in);");
    e.line("    while (L.sb < MK_SB_DONE) mk_run(L.sb, L, budget, slots, sstride, 0u, L.steps);");
    e.line("    *steps_out = L.steps;");
    e.line("    *status_out = L.st;");
    e.line("    return L.outv;");
    e.line("}");
}

} // namespace

uint32_t jit_lds_slot_count(uint32_t nslots, bool heavy, const JitLimits &lim)
{
    if (jit_slots_in_lds(nslots, heavy, lim)) return nslots;
    if (!lim.lds_split || !heavy || !nslots || lim.slot_layout == 0) return 0;
    if (lim.slot_layout < 0 && nslots > kJitWaveBlockedSlots) return 0; // lane-major layout: no split
    // as many slots as fit the LDS budget in 2 KiB allocation granules
    const uint64_t cap = std::min<uint64_t>(lim.lds_slot_bytes, 160u * 1024u);
    const uint32_t n = (uint32_t)(cap / 2048u * 8u);
    // only when LDS takes most of the slots (r02as, 256K lanes: C4 D=400,
    // 320 of 337 slots in LDS, 798 -> 574 us; D=640, 320 of 577, 1,472 ->
    // 1,664 us; D=1024 2,763 -> 3,000 us)
    return n < nslots && (uint64_t)n * 100u >= (uint64_t)nslots * lim.lds_split ? n : 0;
}

bool jit_slots_in_lds(uint32_t nslots, bool heavy, const JitLimits &lim)
{
    // one workgroup may hold at most the CU's 160 KiB of LDS
    const uint64_t cap = std::min<uint64_t>(lim.lds_slot_bytes, 160u * 1024u);
    return heavy && nslots && lim.slot_layout != 0 && (uint64_t)nslots * 256u <= cap;
}

bool jit_lane_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why, JitShape *shape,
                     uint64_t *max_steps, bool *heavy, bool checked, uint32_t *pool)
{
    Graph g;
    if (!analyze(p, lim, g, why)) return false;
    Emitter e;
    const JitShape s = lim.force_stream ? JIT_STREAM : (lim.force_machine || g.cyclic) ? JIT_MACHINE : JIT_STREAM;
    if (pool) {
        // lane pool of the machine shape: slots per wave from the parked state size
        size_t used = 0;
        for (uint32_t r = 0; r < p.nregs; ++r) used += g.used_reg[r] ? 1 : 0;
        const size_t bytes = 8 * used + 16;
        uint32_t m = 0;
        if (s == JIT_MACHINE) {
            if (lim.pool >= 64) { // LDS pool of that many slots per wave
                m = lim.pool / 64 * 64;
                if (g.entry.size() > kJitPoolMaxVariants || m > 4096 || bytes * m > 65536) m = 0;
            } else if (lim.pool >= 2 && lim.pool <= 8) { // K lanes per thread
                m = lim.pool;
            }
        }
        *pool = m;
    }
    if (s == JIT_MACHINE) {
        emit_machine_lane(p, g, e);
    } else {
        narrow_regs(g);
        emit_stream(p, g, e, max_fast_steps(p, g), checked);
    }
    if (!checked && e.s.size() > lim.max_src_bytes) {
        why = "lane source of " + std::to_string(e.s.size()) + " B exceeds the native tier's compile bound (" +
              std::to_string(lim.max_src_bytes) + " B)";
        return false;
    }
    if (shape) *shape = s;
    if (max_steps) *max_steps = s == JIT_STREAM ? max_fast_steps(p, g) : UINT64_MAX;
    if (heavy) *heavy = g.ndops > lim.heavy_ops;
    src = std::move(e.s);
    return true;
}

// Kernel of the stream shape.  A block takes tiles of 4 x 256 contiguous
// inputs (grid-stride); thread tid owns inputs tile*1024 + tid*4 .. +3,
// loads the next tile's 16 bytes before running the current 4 lanes one
// after another, and writes 16 B of out + 4 B of status per tile (+16 B of
// steps on request).  Counters fold per wave (stats_reduce).
// Counters of the stream kernels (the per-wave rows of write_partials /
// add_partials): the step sum per thread, the statuses by ballots in
// wave-uniform registers -- a lane costs a compare per status kind instead of
// count_lane's seven 64-bit adds, which made the counting launches of the
// light kernel VALU-bound (C3: 16.8 vs 12.2 us per launch, r04i).  Called in
// wave-uniform control flow, once per lane slot (`live`: the slot holds an
// input), so the ballots see every lane of the wave.
static const char *const kStreamCount = R"(
struct MkCount {
    unsigned long long steps;                  // per thread
    uint32_t out, done, qu, bu, ov, os;        // wave-uniform
};
__device__ __forceinline__ void mk_count(MkCount &c, bool live, uint32_t steps, uint32_t st)
{
    const uint32_t r = live ? (st & MK_ST_REASON_MASK) : 0u;
    c.steps += live ? steps : 0u;
    c.done += (uint32_t)__popcll(__ballot(live));
    c.out += (uint32_t)__popcll(__ballot(live && (st & MK_ST_HAS_OUTPUT)));
    c.qu += (uint32_t)__popcll(__ballot(r == MK_ST_QUIESCENT));
    if (__ballot(live && r != MK_ST_QUIESCENT)) { // the other ends, counted where they occur
        c.bu += (uint32_t)__popcll(__ballot(r == MK_ST_BUDGET));
        c.ov += (uint32_t)__popcll(__ballot(r == MK_ST_STACK_OVERFLOW));
        c.os += (uint32_t)__popcll(__ballot(r == MK_ST_OUTPUT_STOP));
    }
}
// The wave's row: its own (gid >> 6), or row (gid >> 6) % rows added atomically.
__device__ __forceinline__ void mk_count_store(unsigned long long *partials, uint32_t rows, uint64_t gid,
                                               const MkCount &c)
{
    const unsigned long long s = wave_sum(c.steps);
    if ((gid & 63) != 0) return;
    const unsigned long long v[7] = {s, c.out, c.done, c.qu, c.bu, c.ov, c.os};
    if (!rows) {
        unsigned long long *q = partials + (gid >> 6) * 8;
        for (int k = 0; k < 7; k++) q[k] += v[k];
    } else {
        unsigned long long *q = partials + ((gid >> 6) % rows) * 8;
        for (int k = 0; k < 7; k++)
            if (v[k]) atomicAdd(q + k, v[k]);
    }
}
)";

static const char *const kStreamKernel = R"(
__device__ __forceinline__ void mk_load4(const SParams &p, uint64_t base, int32_t &a, int32_t &b, int32_t &c, int32_t &d)
{
    if (p.io_vec && base + 4 <= p.n) {
        const int4 q = *reinterpret_cast<const int4 *>((const int32_t *)p.in_data + base);
        a = q.x, b = q.y, c = q.z, d = q.w;
        return;
    }
    a = base < p.n ? sched_input(p, base) : 0;
    b = base + 1 < p.n ? sched_input(p, base + 1) : 0;
    c = base + 2 < p.n ? sched_input(p, base + 2) : 0;
    d = base + 3 < p.n ? sched_input(p, base + 3) : 0;
}

extern "C" __global__ void __launch_bounds__(256) mk_jit_exec(SParams p)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + tid;
    const uint64_t tile = 1024u, ntiles = (p.n + tile - 1) / tile;
    MkCount cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    int32_t *slots = p.slots ? p.slots + gid : (int32_t *)0;
    int32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
    uint64_t t = blockIdx.x;
    if (t < ntiles) mk_load4(p, t * tile + (uint64_t)tid * 4u, x0, x1, x2, x3);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * tile + (uint64_t)tid * 4u;
        const int32_t c0 = x0, c1 = x1, c2 = x2, c3 = x3;
        if (t + gridDim.x < ntiles) mk_load4(p, base + (uint64_t)gridDim.x * tile, x0, x1, x2, x3);
        uint32_t s0, s1, s2, s3, t0, t1, t2, t3;
        int32_t o0 = mk_lane_ng(c0, p.budget, slots, p.lanes, &s0, &t0);
        int32_t o1 = mk_lane_ng(c1, p.budget, slots, p.lanes, &s1, &t1);
        int32_t o2 = mk_lane_ng(c2, p.budget, slots, p.lanes, &s2, &t2);
        int32_t o3 = mk_lane_ng(c3, p.budget, slots, p.lanes, &s3, &t3);
        o0 = (t0 & MK_ST_HAS_OUTPUT) ? o0 : 0;
        o1 = (t1 & MK_ST_HAS_OUTPUT) ? o1 : 0;
        o2 = (t2 & MK_ST_HAS_OUTPUT) ? o2 : 0;
        o3 = (t3 & MK_ST_HAS_OUTPUT) ? o3 : 0;
        if (p.io_vec && base + 4 <= p.n) {
            MK_IO_ST(reinterpret_cast<mk_i32x4 *>(p.out + base), (mk_i32x4{o0, o1, o2, o3}));
            MK_IO_ST(reinterpret_cast<uint32_t *>(p.status + base),
                     (t0 & 0xffu) | (t1 & 0xffu) << 8 | (t2 & 0xffu) << 16 | t3 << 24);
            if (p.steps) *reinterpret_cast<uint4 *>(p.steps + base) = make_uint4(s0, s1, s2, s3);
        } else {
            const int32_t ov[4] = {o0, o1, o2, o3};
            const uint32_t sv[4] = {s0, s1, s2, s3}, tv[4] = {t0, t1, t2, t3};
            for (int k = 0; k < 4; ++k) {
                if (base + k >= p.n) break;
                p.out[base + k] = ov[k];
                p.status[base + k] = (uint8_t)tv[k];
                if (p.steps) p.steps[base + k] = sv[k];
            }
        }
        if (p.partials) {
            mk_count(cnt, base < p.n, s0, t0);
            mk_count(cnt, base + 1 < p.n, s1, t1);
            mk_count(cnt, base + 2 < p.n, s2, t2);
            mk_count(cnt, base + 3 < p.n, s3, t3);
        }
    }
    if (p.partials) mk_count_store(p.partials, 0u, gid, cnt);
}

)";

// Kernel of the stream shape for heavy lanes (more than kJitHeavyOps
// micro-ops: long programs, deep stacks): one lane per thread, small blocks
// so that modest batches still spread over every CU, and one copy of the
// lane code (hiprtc time grows with it).  No grid-stride loop: around a
// lane this long, LLVM hoists the slot addresses of the whole program out
// of the loop (C4 d1024: 410 VGPRs, one wave per SIMD, vs 50 without the
// loop); the executor launches one thread per input instead, in chunks
// bounded by the slot memory they need (kJitSlotBytes).
static const char *const kStreamKernelHeavy = R"(
#ifndef MK_HBM_NSLOTS
#define MK_HBM_NSLOTS MK_NSLOTS // slots per lane in the HBM block (all but the LDS-split ones)
#endif
extern "C" __global__ void __launch_bounds__(64) mk_jit_exec(SParams p)
{
    const uint64_t gid = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    uint32_t s = 0u, t = 0u;
    if (gid < p.n) {
#if MK_SLOTS_WAVE_BLOCKED
        // the wave's 64 lanes of slot k are 256 contiguous bytes and its slots
        // follow one another: a wave's stacks are one block (tis_jit.h)
#if MK_SLOTS_BUFFER
        // the wave's block; MK_SLOT_ST/LD add the lane's offset
        int32_t *slots = p.slots ? p.slots + (uint64_t)blockIdx.x * (64ull * MK_HBM_NSLOTS) : (int32_t *)0;
#else
        int32_t *slots = p.slots ? p.slots + (gid >> 6) * (64ull * MK_HBM_NSLOTS) + (gid & 63u) : (int32_t *)0;
#endif
        const int32_t o = mk_lane_ng(sched_input(p, gid), p.budget, slots, 64u, &s, &t);
#else
        const int32_t o = mk_lane_ng(sched_input(p, gid), p.budget, p.slots ? p.slots + gid : (int32_t *)0,
                                     p.lanes, &s, &t);
#endif
        p.out[gid] = (t & MK_ST_HAS_OUTPUT) ? o : 0;
        p.status[gid] = (uint8_t)t;
        if (p.steps) p.steps[gid] = s;
    }
    if (p.partials) {
        MkCount cnt = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
        mk_count(cnt, gid < p.n, s, t);
        mk_count_store(p.partials, p.part_rows ? p.part_rows : 1u, gid, cnt);
    }
}
)";

// Kernel of the machine shape.  Thread gid runs inputs gid, gid + lanes, ...
// one at a time as an MkLane.  Each turn of the wave loop:
//   1. lanes that ended (MK_SB_DONE) write their result and take their next
//      input (prefetched one ahead) -- in bulk, once at least `refill` of the
//      wave's lanes are waiting or nothing else can run;
//   2. the superblock of the wave's lowest running lane is run for every lane
//      sitting on it (a scalar switch on a wave-uniform id).
// A self-loop keeps iterating while enough of its lanes stay in it
// (MK_LOOP_NEED), so that a few long trips do not hold the whole wave.
// The policy word `pol` = refill | loop_num << 8 | loop_min << 16: a loop
// leaves once fewer than loop_num/16 of the lanes it started with remain,
// for groups of at least loop_min lanes.
static const char *const kMachineKernel = R"(
extern "C" __global__ void __launch_bounds__(256) mk_jit_exec(SParams p)
{
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t stride = p.lanes;
    const uint32_t pol = MK_POLICY;
    const uint32_t refill_t = pol & 0xffu;
    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
    int32_t *slots = p.slots ? p.slots + gid : (int32_t *)0;
    // lane j answers input ord(j): the identity, or (p.order) the inputs
    // grouped by value, so that a wave's lanes have similar loop trip counts
#define MK_ORD(j) (p.order ? (uint64_t)p.order[j] : (j))
    uint64_t idx = gid;
    MkLane L;
    mk_init(L, idx < p.n ? sched_input(p, MK_ORD(idx)) : 0);
    if (idx >= p.n) L.sb = MK_SB_IDLE;
    int32_t nxt = idx + stride < p.n ? sched_input(p, MK_ORD(idx + stride)) : 0;
    for (;;) {
        const bool fin = L.sb == MK_SB_DONE;
        const unsigned long long finb = __ballot(fin);
        unsigned long long actb = __ballot(L.sb < MK_SB_DONE);
        if (finb && (!actb || (uint32_t)__popcll(finb) >= refill_t)) {
            if (fin) {
                const uint64_t at = MK_ORD(idx);
                p.out[at] = (L.st & MK_ST_HAS_OUTPUT) ? L.outv : 0;
                p.status[at] = (uint8_t)L.st;
                if (p.steps) p.steps[at] = L.steps;
                count_lane(cnt, L.steps, L.st);
                idx += stride;
                if (idx < p.n) {
                    mk_init(L, nxt);
                    nxt = idx + stride < p.n ? sched_input(p, MK_ORD(idx + stride)) : 0;
                } else {
                    L.sb = MK_SB_IDLE;
                }
            }
            actb = __ballot(L.sb < MK_SB_DONE);
        }
        if (!actb) {
            if (!finb) break;
            continue;
        }
        const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)L.sb, (int)__builtin_ctzll(actb));
        // loop variants: the group's largest step count (exec is full here,
        // as the DPP reduction needs; u is uniform)
        const uint32_t smax = mk_is_loop(u) ? MK_WAVE_MAX(L.sb == u ? L.steps : 0u) : 0u;
        const uint32_t us = MK_SCALAR(u); // the switch value, out of GVN's reach (MK_JIT_UNIFORM_SW)
        if (L.sb == u) mk_run(us, L, p.budget, slots, stride, pol, smax);
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}
)";

// Kernel of the machine shape with lanes grouped by value inside a tile.
// A block takes tiles of MK_TS_T = 256 R contiguous inputs (grid-stride):
//   1. loads them (coalesced: thread t holds inputs t, t + 256, ...) and
//      buckets them by value in LDS: block min / max, 256 buckets of equal
//      width (a power of two), an LDS histogram, its prefix sum and a
//      scatter of (position, input) pairs, one 64-bit word each -- a
//      counting sort whose order inside a bucket does not matter;
//   2. runs them in sorted order, 64 at a time per wave (R rounds, the
//      waves' chunks in snake order so that each wave's chunks balance),
//      every chunk by sweeps then generations (mk_run on the superblock of
//      the lowest running lane until every lane of the chunk has ended); each
//      lane stores its out / status / steps straight to its input's position
//      (the tile's 4 KiB of outputs are whole lines in L2 before they leave).
// Equal inputs take identical paths, and where trip counts follow the input
// (C5's countdowns, the census classes' push loops) a chunk's lanes leave
// their loops together: the idle lanes of generations over unsorted inputs
// (a wave runs each loop for its longest trip) mostly go away, without the
// global sort's atomics and scattered result writes (MK_JIT_ORDER).
// LDS bank conflicts come only from operations at data-dependent addresses
// (the histogram and rank atomics, the scatter); round 6 halved them per
// input (7 -> 3: no results through LDS, one 64-bit scatter in place of a
// 32- and a 16-bit one) and made the scatter of equal or presorted inputs
// conflict-free (the strided layout; R consecutive inputs per thread made it
// 4-way).
static const char *const kMachineSortKernel = R"(
extern "C" __device__ uint32_t __ockl_wfscan_add_u32(uint32_t, bool);
// a chunk's end reasons: the lanes that ended, those quiescent, and the
// three other reasons only when some lane ended otherwise (round 6)
#define MK_TS_COUNT_REASONS(live, rs)                                                            \
    do {                                                                                         \
        const unsigned long long lv_ = __ballot(live), qu_ = __ballot((rs) == MK_ST_QUIESCENT);  \
        c_done += (uint32_t)__popcll(lv_);                                                       \
        c_qu += (uint32_t)__popcll(qu_);                                                         \
        if (lv_ & ~qu_) {                                                                        \
            c_bu += (uint32_t)__popcll(__ballot((rs) == MK_ST_BUDGET));                          \
            c_ov += (uint32_t)__popcll(__ballot((rs) == MK_ST_STACK_OVERFLOW));                  \
            c_os += (uint32_t)__popcll(__ballot((rs) == MK_ST_OUTPUT_STOP));                     \
        }                                                                                        \
    } while (0)
#define MK_TS_T (256u * MK_TS_R)
#define MK_TS_NB 256u
extern "C" __global__ void __launch_bounds__(256) mk_jit_exec(SParams p)
{
    __shared__ uint64_t s_kp[MK_TS_T]; // the tile in sorted order: position << 32 | input
    __shared__ __attribute__((aligned(16))) uint32_t s_cnt[MK_TS_NB]; // bucket counts
    __shared__ __attribute__((aligned(16))) uint32_t s_cur[MK_TS_NB]; // bucket cursors (ranks)
    __shared__ uint32_t s_red[8];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + tid;
    const uint32_t pol = MK_POLICY;
    // counters: steps per lane (one wave sum at the end), the others
    // wave-uniform (scalar registers): outputs, lanes, and the four end reasons
    uint64_t c_steps = 0u;
    uint32_t c_out = 0u, c_done = 0u, c_qu = 0u, c_bu = 0u, c_ov = 0u, c_os = 0u;
    // stack slots lane-major ([slot][lanes]: a slot row of all resident
    // lanes is contiguous; wave-blocked rows measured slower here, round 6:
    // t1_two_stacks 236 -> 266 us, t2_dyn_depth 120 -> 123 us, r08n)
    int32_t *slots = p.slots ? p.slots + gid : (int32_t *)0;
#if MK_PROF
    // MK_JIT_PROF: shader-clock cycles per phase, per wave, in place of the
    // counters (tools/probe/c5_decomp.py reads them from the stats)
    const uint64_t pf_t0 = MK_T();
    uint64_t pf_sort = 0u, pf_chunk = 0u, pf_loop = 0u, pf_other = 0u, pf_rounds = 0u, pf_lrounds = 0u;
#endif
    const uint64_t ntiles = (p.n + MK_TS_T - 1) / MK_TS_T;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * MK_TS_T;
        const uint32_t m = p.n - base < MK_TS_T ? (uint32_t)(p.n - base) : MK_TS_T;
#if MK_PROF
        uint64_t pf_a = MK_T();
#endif
        // 1. inputs tid + 256 k of the tile, their range
        int32_t v[MK_TS_R];
        if (p.io_vec && m == MK_TS_T) {
            for (uint32_t k = 0; k < MK_TS_R; ++k) v[k] = ((const int32_t *)p.in_data)[base + tid + 256u * k];
        } else {
            for (uint32_t k = 0; k < MK_TS_R; ++k) v[k] = tid + 256u * k < m ? sched_input(p, base + tid + 256u * k) : 0;
        }
        uint32_t lo = 0xFFFFFFFFu, hi = 0u; // biased: signed order as unsigned
        for (uint32_t k = 0; k < MK_TS_R; ++k) {
            if (tid + 256u * k >= m) continue;
            const uint32_t b = (uint32_t)v[k] ^ 0x80000000u;
            lo = b < lo ? b : lo;
            hi = b > hi ? b : hi;
        }
        s_cnt[tid] = 0u;
        lo = MK_WAVE_MIN(lo);
        hi = MK_WAVE_MAX(hi);
        if (lane == 0u) {
            s_red[wave] = lo;
            s_red[4u + wave] = hi;
        }
        __syncthreads();
        for (uint32_t w = 0; w < 4u; ++w) {
            lo = s_red[w] < lo ? s_red[w] : lo;
            hi = s_red[4u + w] > hi ? s_red[4u + w] : hi;
        }
        // bucket = (x - lo) >> sh, sh the smallest shift that fits the range into 256 buckets
        const uint32_t span = hi - lo;
        const uint32_t bits = span ? 32u - (uint32_t)__clz(span) : 0u;
        const uint32_t sh = bits > 8u ? bits - 8u : 0u;
        uint32_t bk[MK_TS_R];
        for (uint32_t k = 0; k < MK_TS_R; ++k) {
            // a tile of one value (span 0) goes by position, bucket tid: its
            // inputs' atomics on one bucket would serialize (C5 with every
            // input 0 spent half its time here, profiles/r04r_c5_phase_prof.jsonl)
            bk[k] = span ? (((uint32_t)v[k] ^ 0x80000000u) - lo) >> sh : tid;
            if (tid + 256u * k < m) atomicAdd(&s_cnt[bk[k]], 1u);
        }
        __syncthreads();
        // the buckets' cursors, an exclusive prefix sum of the counts (thread
        // tid owns bucket tid): a DPP wave scan (round 6; six __shfl_up steps
        // were six LDS permute round trips) and the waves' totals.  Every
        // wave scanning all 256 counts instead (one barrier fewer) measured
        // level on C5 but 12% slower on the JRO-heavy census class
        // (profiles/r08_c5_sort_ab.txt, r08al)
        {
            const uint32_t c = s_cnt[tid];
            const uint32_t x = __ockl_wfscan_add_u32(c, true);
            if (lane == 63u) s_red[wave] = x;
            __syncthreads();
            uint32_t pre = 0u;
            for (uint32_t w = 0; w < wave; ++w) pre += s_red[w];
            s_cur[tid] = pre + x - c;
            __syncthreads();
        }
        // every rank first, then the scatter: the atomics' round trips overlap
        uint32_t d[MK_TS_R];
        for (uint32_t k = 0; k < MK_TS_R; ++k)
            d[k] = tid + 256u * k < m ? atomicAdd(&s_cur[bk[k]], 1u) : 0u;
        for (uint32_t k = 0; k < MK_TS_R; ++k)
            if (tid + 256u * k < m) s_kp[d[k]] = (uint64_t)(tid + 256u * k) << 32 | (uint32_t)v[k];
        __syncthreads();
#if MK_PROF
        pf_sort += MK_T() - pf_a;
        pf_a = MK_T();
#endif
        // 2. the sorted lanes, 64 per chunk, each wave's chunks in snake order
        // (the next tile's first barrier keeps s_kp until every wave is done)
#if defined(MK_PAIR)
        // two lanes per thread: a pair of adjacent sorted chunks, the pairs
        // in snake order.  One sweep pass serves both lanes (a variant's
        // ballot, its skip when neither lane is on it); the loops still run
        // one lane at a time: a paired countdown (two interleaved dependency
        // chains, measured round 6) did 6% more decrements, 2 x max(A, B)
        // against A + B, without a faster rate (profiles/r08_c5_sort_ab.txt)
        for (uint32_t r = 0; r < MK_TS_R; r += 2u) {
            const uint32_t q = (r >> 1) * 4u + (((r >> 1) & 1u) ? 3u - wave : wave);
            const uint32_t jA = q * 128u + lane, jB = jA + 64u;
            const bool liveA = jA < m, liveB = jB < m;
            uint64_t kpA = liveA ? s_kp[jA] : 0u;
            const uint64_t kpB = liveB ? s_kp[jB] : 0u;
            MkLane A, B;
            mk_init(A, (int32_t)(uint32_t)kpA);
            mk_init(B, (int32_t)(uint32_t)kpB);
            if (!liveA) A.sb = MK_SB_IDLE;
            if (!liveB) B.sb = MK_SB_IDLE;
#if defined(MK_SWEEP_LIST)
#define MK_SWEEP_STEP(v, loop)                                                                   \
            if (__ballot(A.sb == (v) || B.sb == (v))) {                                              \
                /* one wave maximum for both lanes (an upper bound for each: */                      \
                /* a loop's fast phase is only shortened by it) */                                   \
                const uint32_t sa_ = A.sb == (v) ? A.steps : 0u, sb_ = B.sb == (v) ? B.steps : 0u;   \
                const uint32_t sm_ = (loop) ? MK_WAVE_MAX(sa_ > sb_ ? sa_ : sb_) : 0u;               \
                if (A.sb == (v)) mk_run((v), A, p.budget, slots, p.lanes, pol, sm_);                 \
                if (B.sb == (v)) mk_run((v), B, p.budget, slots, p.lanes, pol, sm_);                 \
            }
            MK_SWEEP_LIST(MK_SWEEP_STEP)
#if defined(MK_SWEEP_COLD)
            if (__ballot((A.sb < 64u && ((MK_SWEEP_COLD_MASK >> A.sb) & 1ull)) ||
                         (B.sb < 64u && ((MK_SWEEP_COLD_MASK >> B.sb) & 1ull)))) {
                MK_SWEEP_COLD(MK_SWEEP_STEP)
            }
#endif
#undef MK_SWEEP_STEP
#endif
            // what the pass left, lane A then lane B (B moved into A): rounds
            bool live = liveA;
#pragma unroll 1
            for (uint32_t h = 0; h < 2u; ++h) {
                for (;;) {
                    const unsigned long long actb = __ballot(A.sb < MK_SB_DONE);
                    if (!actb) break;
                    const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)A.sb, (int)__builtin_ctzll(actb));
                    const uint32_t smax = mk_is_loop(u) ? MK_WAVE_MAX(A.sb == u ? A.steps : 0u) : 0u;
                    const uint32_t us = MK_SCALAR(u);
                    if (A.sb == u) mk_run(us, A, p.budget, slots, p.lanes, pol, smax);
                }
                if (live) {
                    const uint64_t at = base + (kpA >> 32);
                    p.out[at] = (A.st & MK_ST_HAS_OUTPUT) ? A.outv : 0;
                    p.status[at] = (uint8_t)A.st;
                    if (p.steps) p.steps[at] = A.steps;
                }
                const uint32_t rs = live ? (A.st & MK_ST_REASON_MASK) : 0u;
                c_steps += live ? (uint64_t)A.steps : 0u;
                c_out += (uint32_t)__popcll(__ballot(live && (A.st & MK_ST_HAS_OUTPUT)));
                MK_TS_COUNT_REASONS(live, rs);
                A = B;
                kpA = kpB;
                live = liveB;
            }
        }
#else
        for (uint32_t r = 0; r < MK_TS_R; ++r) {
            const uint32_t c = r * 4u + ((r & 1u) ? 3u - wave : wave);
            const uint32_t j = c * 64u + lane;
            const bool live = j < m;
            const uint64_t kp = live ? s_kp[j] : 0u;
            MkLane L;
            mk_init(L, (int32_t)(uint32_t)kp);
            if (!live) L.sb = MK_SB_IDLE;
#if defined(MK_SWEEP_LIST)
            // sweep dispatch (MK_JIT_SWEEP): the variants in forward order,
            // each run for the lanes on it, skipped by one ballot when none
            // is; MK_SWEEP_PASSES passes, then the rounds below
#define MK_SWEEP_STEP(v, loop)                                                                   \
            if (__ballot(L.sb == (v))) {                                                             \
                const uint32_t smax_ = (loop) ? MK_WAVE_MAX(L.sb == (v) ? L.steps : 0u) : 0u;        \
                if (L.sb == (v)) mk_run((v), L, p.budget, slots, p.lanes, pol, smax_);               \
            }
            for (uint32_t ps = 0; ps < MK_SWEEP_PASSES && __ballot(L.sb < MK_SB_DONE); ++ps) {
                MK_SWEEP_LIST(MK_SWEEP_STEP)
#if defined(MK_SWEEP_COLD)
                if (__ballot(L.sb < 64u && ((MK_SWEEP_COLD_MASK >> L.sb) & 1ull))) {
                    MK_SWEEP_COLD(MK_SWEEP_STEP)
                }
#endif
            }
#undef MK_SWEEP_STEP
#endif
            // rounds: the lowest lane's variant at a time (after the sweep
            // passes, for the lanes they left: loops over several variants)
            for (;;) {
                const unsigned long long actb = __ballot(L.sb < MK_SB_DONE);
                if (!actb) break;
                const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)L.sb, (int)__builtin_ctzll(actb));
#if MK_PROF
                const uint64_t pf_r = MK_T();
#endif
                const uint32_t smax = mk_is_loop(u) ? MK_WAVE_MAX(L.sb == u ? L.steps : 0u) : 0u;
                const uint32_t us = MK_SCALAR(u); // the switch value, out of GVN's reach (MK_JIT_UNIFORM_SW)
                if (L.sb == u) mk_run(us, L, p.budget, slots, p.lanes, pol, smax);
#if MK_PROF
                const uint64_t pf_d = MK_T() - pf_r;
                if (mk_is_loop(u)) pf_loop += pf_d, ++pf_lrounds;
                else pf_other += pf_d;
                ++pf_rounds;
#endif
            }
            if (live) {
                const uint64_t at = base + (kp >> 32);
                p.out[at] = (L.st & MK_ST_HAS_OUTPUT) ? L.outv : 0;
                p.status[at] = (uint8_t)L.st;
                if (p.steps) p.steps[at] = L.steps;
            }
            const uint32_t rs = live ? (L.st & MK_ST_REASON_MASK) : 0u;
            c_steps += live ? (uint64_t)L.steps : 0u;
            c_out += (uint32_t)__popcll(__ballot(live && (L.st & MK_ST_HAS_OUTPUT)));
            MK_TS_COUNT_REASONS(live, rs);
        }
#endif
#if MK_PROF
        pf_chunk += MK_T() - pf_a;
#endif
    }
#if MK_PROF
    if (p.partials && lane == 0u) {
        unsigned long long *q = p.partials + (gid >> 6) * 8u;
        q[0] += MK_T() - pf_t0;
        q[1] += pf_sort;
        q[2] += pf_chunk;
        q[3] += pf_loop;
        q[4] += pf_other;
        q[5] += 0u; // (no results phase since round 6)
        q[6] += pf_rounds;
        q[7] += pf_lrounds;
    }
    (void)c_steps; (void)c_out; (void)c_done; (void)c_qu; (void)c_bu; (void)c_ov; (void)c_os;
#else
    c_steps = wave_sum(c_steps); // whole wave active: the tile loop's bound is uniform
    if (p.partials && lane == 0u) { // this wave's row (write_partials' layout)
        unsigned long long *q = p.partials + (gid >> 6) * 8u;
        q[0] += c_steps;
        q[1] += c_out;
        q[2] += c_done;
        q[3] += c_qu;
        q[4] += c_bu;
        q[5] += c_ov;
        q[6] += c_os;
    }
#endif
}
)";


JitLimits JitLimits::from_env()
{
    JitLimits l;
    auto num = [](const char *name, auto &v) {
        const char *s = std::getenv(name);
        if (s && *s) v = (std::remove_reference_t<decltype(v)>)std::strtoull(s, nullptr, 10);
    };
    auto flag = [](const char *name, bool &v) {
        const char *s = std::getenv(name);
        if (s && *s) v = s[0] == '1';
    };
    if (const char *s = std::getenv("MK_JIT"); s && !std::strcmp(s, "0")) l.disabled = true;
    if (const char *s = std::getenv("MK_JIT_SHAPE")) {
        l.force_machine = !std::strcmp(s, "machine");
        l.force_stream = !std::strcmp(s, "stream");
    }
    if (const char *s = std::getenv("MK_JIT_POLICY")) {
        unsigned r = 0, nu = 0, mi = 0;
        if (std::sscanf(s, "%u,%u,%u", &r, &nu, &mi) == 3 && r <= 64 && nu <= 16 && mi <= 64)
            l.policy = r | nu << 8 | mi << 16;
    }
    if (const char *s = std::getenv("MK_JIT_SLOT_LAYOUT"))
        l.slot_layout = !std::strcmp(s, "blocked") ? 1 : !std::strcmp(s, "lane") ? 0 : -1;
    if (const char *s = std::getenv("MK_JIT_COMPILE_S"); s && *s) l.max_compile_s = std::strtod(s, nullptr);
    num("MK_JIT_MAX_DOPS", l.max_dops);
    num("MK_JIT_MAX_SRC", l.max_src_bytes);
    num("MK_JIT_LOOP_UNROLL", l.loop_unroll);
    num("MK_JIT_PREFETCH", l.prefetch);
    num("MK_JIT_HEAVY_OPS", l.heavy_ops);
    num("MK_JIT_SLOT_BYTES", l.slot_bytes);
    if (!l.slot_bytes) l.slot_bytes = kJitSlotBytes;
    num("MK_JIT_POOL", l.pool);
    flag("MK_JIT_ORDER", l.order);
    flag("MK_JIT_TILE_SORT", l.tile_sort);
    num("MK_JIT_TS_ROUNDS", l.ts_rounds);
    if (const char *v = std::getenv("MK_JIT_LDS_SLOTS"); v && *v) {
        l.lds_slot_bytes = (size_t)std::strtoull(v, nullptr, 10);
        l.lds_auto = false;
    }
    num("MK_JIT_SAT_BLOCK", l.sat_block);
    if (l.sat_block != 4 && l.sat_block != 8 && l.sat_block != 16 && l.sat_block != 32) l.sat_block = 4;
    num("MK_JIT_VGPR_FILE", l.vgpr_file);
    flag("MK_JIT_PAIR", l.pair);
    flag("MK_JIT_TUNE_GRID", l.tune_grid);
    if (!l.vgpr_file || l.vgpr_file > 512) l.vgpr_file = 512;
    flag("MK_JIT_SWEEP", l.sweep);
    flag("MK_JIT_SAT_COUNT", l.sat_count);
    flag("MK_JIT_TUNE_REGS", l.tune_regs);
    num("MK_JIT_LDS_SPLIT", l.lds_split);
    flag("MK_JIT_PROF", l.prof);
    if (l.ts_rounds != 0 && l.ts_rounds != 1 && l.ts_rounds != 2 && l.ts_rounds != 4 && l.ts_rounds != 8 && l.ts_rounds != 16)
        l.ts_rounds = 0;
    num("MK_JIT_TS_ROUNDS_SLOTS", l.ts_rounds_slots);
    if (l.ts_rounds_slots > 16 || (l.ts_rounds_slots & (l.ts_rounds_slots - 1))) l.ts_rounds_slots = 2;
    return l;
}

std::string JitLimits::key() const
{
    char b[256];
    snprintf(b, sizeof b,
             "shape=%s,policy=%08x,dops=%zu,src=%zu,unroll=%d,layout=%d,pf=%zu,heavy=%zu,pool=%u,order=%d,"
             "tsort=%d,tsr=%u,lds=%zu%s,tune=%d,split=%u,sblk=%u",
             force_machine ? "machine" : force_stream ? "stream" : "auto", policy, max_dops, max_src_bytes,
             loop_unroll, slot_layout, prefetch, heavy_ops, pool, (int)order,
             (int)tile_sort, ts_rounds, lds_slot_bytes, lds_auto ? "auto" : "",
             (int)tune_regs, lds_split, sat_block);
    std::string k = b;
    if (!sat_count) k += ",scount=0";
    if (!sweep) k += ",sweep=0";
    if (prof) k += ",prof=1";
    if (vgpr_file != 512) k += ",vfile=" + std::to_string(vgpr_file);
    if (!pair) k += ",pair=0";
    if (!tune_grid) k += ",tgrid=0";
    if (ts_rounds_slots != 2) k += ",tsrs=" + std::to_string(ts_rounds_slots);
    return k;
}

// Kernel of the machine shape with lane compaction.  One wave per block,
// owning a pool of MK_POOL parked lanes in LDS (MkPool: registers,
// superblock, steps, input index) and a histogram of how many parked lanes
// sit on each superblock variant.  Each turn:
//   1. free slots take new inputs, 64 at a time (chunks of 64 inputs dealt
//      round-robin over the waves);
//   2. the variant u with the most parked lanes is chosen, and up to 64 of
//      its lanes are claimed into registers (MkLane, one per thread);
//   3. mk_run(u) runs them together.  A lane that left u is parked again on
//      its new variant, or, at MK_SB_DONE, answers its input and frees its
//      slot.  For a self-loop (mk_is_loop) the loop leaves once a quarter of
//      its lanes have left (MK_LOOP_NEED), and the group is topped up from
//      the lanes parked on u and run again -- as long as it is no smaller
//      than the largest group parked elsewhere; otherwise its lanes are
//      parked (still on u, at an iteration boundary) and the turn ends.
// So the lanes of a data-dependent loop stay together whatever their trip
// counts: a lane that leaves is replaced by one waiting at the loop head,
// instead of idling (predicated) until the group's longest trip ends.
// Stack slots belong to pool slots (column wave * MK_POOL + slot, stride
// p.lanes = waves * MK_POOL), so a lane's stacks follow it between threads.
static const char *const kMachinePoolKernel = R"(
#define MK_SLOT_FREE 0xFFFFFFFFu
#define MK_SLOT_BUSY 0xFFFFFFFDu
#define MK_NONE 0xFFFFFFFFu
MK_FN uint32_t mk_rank(unsigned long long b)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
MK_FN void mk_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
// Whole wave: each lane with `want` gets a distinct pool slot whose sb is
// `key` (the lane of rank r among the wanting lanes the r-th such slot), or
// MK_NONE when there are fewer such slots; *got = slots handed out.
MK_FN uint32_t mk_claim(const uint32_t *sb, uint32_t *xfer, uint32_t key, bool want, uint32_t &got)
{
    const uint32_t lane = threadIdx.x;
    const unsigned long long wb = __ballot(want);
    const uint32_t nwant = (uint32_t)__popcll(wb);
    uint32_t found = 0u;
    for (uint32_t base = 0u; base < MK_POOL && found < nwant; base += 64u) {
        const uint32_t s = base + lane;
        const bool m = sb[s] == key;
        const unsigned long long mb = __ballot(m);
        const uint32_t k = found + mk_rank(mb);
        if (m && k < nwant) xfer[k] = s;
        found += (uint32_t)__popcll(mb);
    }
    mk_wave_sync();
    got = found < nwant ? found : nwant;
    const uint32_t r = mk_rank(wb);
    const uint32_t s = want && r < got ? xfer[r] : MK_NONE;
    mk_wave_sync();
    return s;
}
// Whole wave: (count << 16 | (0xFFFF - v)) of the variant with the most parked lanes.
MK_FN uint32_t mk_pick(const uint32_t *hist)
{
    uint32_t best = 0u;
    for (uint32_t v = threadIdx.x; v < MK_NV; v += 64u) {
        const uint32_t c = hist[v];
        const uint32_t key = c ? (c << 16) | (0xFFFFu - v) : 0u;
        best = key > best ? key : best;
    }
    return MK_WAVE_MAX(best);
}

extern "C" __global__ void __launch_bounds__(64) mk_jit_exec(SParams p)
{
    __shared__ MkPool P;
    __shared__ uint32_t hist[MK_NV];
    __shared__ uint32_t xfer[64];
    const uint32_t lane = threadIdx.x;
    const uint64_t gw = blockIdx.x, nw = gridDim.x;
    const uint64_t gid = gw * 64u + lane;
    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
    for (uint32_t s = lane; s < MK_POOL; s += 64u) P.sb[s] = MK_SLOT_FREE;
    for (uint32_t v = lane; v < MK_NV; v += 64u) hist[v] = 0u;
    mk_wave_sync();
    uint32_t nfree = MK_POOL;
    uint64_t chunk = gw; // next 64 inputs: [chunk * 64, chunk * 64 + 64)
    int32_t *const sbase = p.slots ? p.slots + gw * (uint64_t)MK_POOL : (int32_t *)0;
    MkLane L;
    mk_init(L, 0);
    uint32_t my = MK_NONE; // pool slot of the lane this thread holds
    uint64_t myidx = 0;
    // retire a held lane that left u: answer its input or park it
    auto leave = [&](const uint32_t u, const bool all) -> uint32_t {
        const bool go = my != MK_NONE && (all || L.sb != u);
        const bool done = go && L.sb == MK_SB_DONE;
        if (done) {
            p.out[myidx] = (L.st & MK_ST_HAS_OUTPUT) ? L.outv : 0;
            p.status[myidx] = (uint8_t)L.st;
            if (p.steps) p.steps[myidx] = L.steps;
            count_lane(cnt, L.steps, L.st);
            P.sb[my] = MK_SLOT_FREE;
        } else if (go) {
            mk_park(P, my, L, myidx);
            atomicAdd(&hist[L.sb], 1u);
        }
        if (go) my = MK_NONE;
        mk_wave_sync();
        return (uint32_t)__popcll(__ballot(done));
    };
    // new inputs into free slots, 64 at a time
    auto fill = [&]() {
        while (nfree >= 64u && chunk * 64u < p.n) {
            const uint64_t i = chunk * 64u + lane;
            const bool has = i < p.n;
            uint32_t got;
            const uint32_t s = mk_claim(P.sb, xfer, MK_SLOT_FREE, has, got);
            if (s != MK_NONE) {
                MkLane F;
                mk_init(F, sched_input(p, i));
                mk_park(P, s, F, i);
            }
            if (lane == 0u) hist[0] += got;
            mk_wave_sync();
            nfree -= got;
            chunk += nw;
        }
    };
    for (;;) {
        fill();
        const uint32_t best = mk_pick(hist);
        if (!(best >> 16)) break; // nothing parked, no inputs left
        const uint32_t u = 0xFFFFu - (best & 0xFFFFu);
        uint32_t got;
        my = mk_claim(P.sb, xfer, u, true, got);
        if (!got) break; // histogram and pool disagree: stop rather than spin (lanes stay unanswered)
        if (my != MK_NONE) {
            mk_unpark(P, my, L, myidx);
            P.sb[my] = MK_SLOT_BUSY;
        }
        if (lane == 0u) hist[u] -= got;
        mk_wave_sync();
        const bool loop = mk_is_loop(u);
        for (;;) {
            // loop variants: the group's largest step count (exec is full here)
            const uint32_t smax = loop ? MK_WAVE_MAX(my != MK_NONE ? L.steps : 0u) : 0u;
            const uint32_t pol = loop ? (12u << 8) | (1u << 16) : 0u; // leave a loop at a quarter gone
            if (my != MK_NONE) mk_run(u, L, p.budget, sbase ? sbase + my : (int32_t *)0, p.lanes, pol, smax);
            if (!loop) {
                nfree += leave(u, true);
                break;
            }
            nfree += leave(u, false);
            fill();
            // top the group up from the lanes parked on u
            uint32_t add;
            const uint32_t s = mk_claim(P.sb, xfer, u, my == MK_NONE, add);
            if (s != MK_NONE) {
                my = s;
                mk_unpark(P, my, L, myidx);
                P.sb[my] = MK_SLOT_BUSY;
            }
            if (lane == 0u) hist[u] -= add;
            mk_wave_sync();
            const uint32_t nin = (uint32_t)__popcll(__ballot(my != MK_NONE));
            if (!nin) break;
            if (nin < (mk_pick(hist) >> 16)) { // a larger group waits elsewhere
                nfree += leave(u, true);
                break;
            }
        }
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}
)";

// Kernel of the machine shape with K lanes per thread (MK_KLANES): lane
// compaction in registers.  Each thread holds MK_KLANES lanes (Q[]); a wave
// turn picks the lowest superblock variant u any of its 64 x K lanes sits on,
// every thread activates one of its lanes on u (if it has one) and mk_run(u)
// runs them together.  For a self-loop the loop leaves once a quarter of the
// group has left (MK_LOOP_NEED), and each thread whose lane left swaps in
// another of its lanes waiting on u; the loop runs on while that keeps at
// least half of the wave busy (or nothing else is runnable).  So a loop's
// lanes are replaced as they finish instead of idling until the wave's
// longest trip ends, with no memory traffic: the swap is a select over K
// register copies.  Lanes that end answer their input; once MK_REFILL_MIN of
// the wave's lanes have ended (or nothing else can run) they take new
// inputs, dealt from the wave's chunks of 64 (chunk c of wave w: w + c*nw).
// Stack slots belong to (thread, lane slot): column gid * K + k, stride
// p.lanes = threads * K.
static const char *const kMachineMultiKernel = R"(
#define MK_REFILL_MIN 64u
#define MK_SB_FREE 0xFFFFFFFDu // answered: the slot waits for a new input
MK_FN uint32_t mk_rank64(unsigned long long b)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}
// The K lane slots are separate variables Q0, Q1, ... (MK_EACH(F) expands
// F(0) F(1) ...): a register array indexed in a loop stays in scratch.
#define MK_GET(j) if (k == j##u) L = Q##j;
#define MK_PUT(j) if (k == j##u) Q##j = L;
#define MK_FIND(j) if (k == MK_KLANES && Q##j.sb == u && j##u != skip) k = j##u;

extern "C" __global__ void __launch_bounds__(256) mk_jit_exec(SParams p)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t gw = gid >> 6, nw = ((uint64_t)gridDim.x * 256u) >> 6;
    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
#define MK_DECL(j) MkLane Q##j; uint64_t qi##j;
    MK_EACH(MK_DECL)
    // the wave's input stream: chunk c of this wave covers [(gw + c*nw) * 64, +64)
    uint64_t spos = 0; // inputs of the wave's stream handed out so far (uniform)
#define MK_IDX(pos) ((gw + ((pos) >> 6) * nw) * 64u + ((pos) & 63u))
#define MK_FIRST(j) { const uint64_t i = MK_IDX(spos + lane); spos += 64u; \
        mk_init(Q##j, i < p.n ? sched_input(p, i) : 0); if (i >= p.n) Q##j.sb = MK_SB_IDLE; qi##j = i; }
    MK_EACH(MK_FIRST)
    int32_t *const sbase = p.slots ? p.slots + gid * MK_KLANES : (int32_t *)0;
    MkLane L;
    mk_init(L, 0);
    for (;;) {
        // retire ended lanes; refill them once enough have ended or nothing else runs
        uint32_t runnable = MK_SB_IDLE, ndone = 0;
#define MK_RETIRE(j) \
        if (Q##j.sb == MK_SB_DONE) { \
            p.out[qi##j] = (Q##j.st & MK_ST_HAS_OUTPUT) ? Q##j.outv : 0; \
            p.status[qi##j] = (uint8_t)Q##j.st; \
            if (p.steps) p.steps[qi##j] = Q##j.steps; \
            count_lane(cnt, Q##j.steps, Q##j.st); \
            Q##j.sb = MK_SB_FREE; \
        } \
        ndone += Q##j.sb == MK_SB_FREE ? 1u : 0u; \
        runnable = Q##j.sb < MK_SB_FREE && Q##j.sb < runnable ? Q##j.sb : runnable;
        MK_EACH(MK_RETIRE)
        const uint32_t wdone = (uint32_t)__builtin_amdgcn_readfirstlane(__ockl_wfred_add_u32(ndone));
        const uint32_t umin = MK_WAVE_MIN(runnable);
        if (wdone && (wdone >= MK_REFILL_MIN || umin >= MK_SB_FREE) && spos < (uint64_t)1 << 62) {
            bool more = false;
#define MK_REFILL(j) { \
            const bool want = Q##j.sb == MK_SB_FREE; \
            const unsigned long long b = __ballot(want); \
            const uint64_t i = MK_IDX(spos + mk_rank64(b)); \
            spos += (uint64_t)__popcll(b); \
            if (want) { \
                if (i < p.n) { mk_init(Q##j, sched_input(p, i)); qi##j = i; } \
                else Q##j.sb = MK_SB_IDLE; \
            } \
            more = more || (want && i < p.n); }
            MK_EACH(MK_REFILL)
            if (!__ballot(more)) spos = (uint64_t)1 << 62; // the wave's stream is exhausted
            continue;
        }
        if (umin >= MK_SB_FREE) break; // nothing runnable, nothing to refill
        const uint32_t u = umin;
        const bool loop = mk_is_loop(u);
        uint32_t k = MK_KLANES, skip = MK_KLANES;
        MK_EACH(MK_FIND)
        bool has = k < MK_KLANES;
        MK_EACH(MK_GET)
        for (;;) {
            // loop variants: the group's largest step count (exec is full here)
            const uint32_t smax = loop ? MK_WAVE_MAX(has ? L.steps : 0u) : 0u;
            const uint32_t pol = (12u << 8) | (1u << 16); // a loop leaves at a quarter of its lanes gone
            if (has) mk_run(u, L, p.budget, sbase ? sbase + k : (int32_t *)0, p.lanes, pol, smax);
            MK_EACH(MK_PUT)
            if (!loop) break;
            // threads whose lane left u swap in another of their lanes on u
            if (has && L.sb != u) {
                skip = k;
                k = MK_KLANES;
                MK_EACH(MK_FIND)
                has = k < MK_KLANES;
                MK_EACH(MK_GET)
            }
            const uint32_t nin = (uint32_t)__popcll(__ballot(has));
            if (nin == 0u) break;
            if (nin < 32u) { // under half the wave: leave if anything else could run
                bool other = false;
#define MK_OTHER(j) other = other || (Q##j.sb != u && Q##j.sb < MK_SB_FREE);
                MK_EACH(MK_OTHER)
                if (__ballot(other)) break;
            }
        }
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}
)";

namespace {
// Everything a module needs before its lane code: types, status codes,
// policy, the flag / loop helpers, the slot-access macros, mk_device_common.
std::string module_prelude(JitShape shape, const JitLimits &lim, uint32_t pool, bool sat, bool narrow_slots = false)
{
    Emitter e;
    if (shape == JIT_MACHINE && pool >= 64) e.line("#define MK_POOL %uu", pool);
    else if (shape == JIT_MACHINE && pool >= 2) {
        e.line("#define MK_KLANES %uu", pool);
        std::string each = "#define MK_EACH(F)";
        for (uint32_t j = 0; j < pool; ++j) each += " F(" + std::to_string(j) + ")";
        e.line("%s", each.c_str());
    }
    // hiprtc declares the fixed-width integer types in __hip_internal only
    e.line("typedef __hip_internal::int8_t int8_t;");
    e.line("typedef __hip_internal::uint8_t uint8_t;");
    e.line("typedef __hip_internal::int16_t int16_t;");
    e.line("typedef __hip_internal::uint16_t uint16_t;");
    e.line("typedef __hip_internal::int32_t int32_t;");
    e.line("typedef __hip_internal::uint32_t uint32_t;");
    e.line("typedef __hip_internal::int64_t int64_t;");
    e.line("typedef __hip_internal::uint64_t uint64_t;");
    e.line("#define MK_IN_I64 %d", MK_IN_I64);
    e.line("#define MK_IN_I32 %d", MK_IN_I32);
    e.line("#define MK_GEN_MASKED %d", MK_GEN_MASKED);
    e.line("#define MK_ST_REASON_MASK %d", MK_ST_REASON_MASK);
    e.line("#define MK_ST_HAS_OUTPUT %d", MK_ST_HAS_OUTPUT);
    e.line("#define MK_ST_QUIESCENT %d", MK_ST_QUIESCENT);
    e.line("#define MK_ST_BUDGET %d", MK_ST_BUDGET);
    e.line("#define MK_ST_STACK_OVERFLOW %d", MK_ST_STACK_OVERFLOW);
    e.line("#define MK_ST_OUTPUT_STOP %d", MK_ST_OUTPUT_STOP);
    e.line("#define MK_FN static __device__ __forceinline__");
    e.line("#define MK_CTABLE static __device__ const");
    // machine-shape policy word, a constant of the module so that the loop
    // exit tests fold (generational: MK_KEEP is "some lane still looping")
    e.line("#define MK_POLICY 0x%08xu", lim.policy);
    if (lim.ts_rounds) // kMachineSortKernel: lanes per thread per tile (else the lane source's choice)
        e.line("#define MK_TS_R %uu", lim.ts_rounds);
    if (shape == JIT_MACHINE) // machine kernels: sweep passes before rounds (stream modules' sources as they were)
        e.line("#define MK_SWEEP_PASSES 1u");
    if (lim.prof) { // kMachineSortKernel: cycles per phase in place of the counters (MK_JIT_PROF)
        e.line("#define MK_PROF 1");
        e.line("#define MK_T() __builtin_amdgcn_s_memtime()");
    }
    e.line("#define MK_ALL(p) (__ballot(!(p)) == 0ull)");
    // MK_JIT_PRIO=1: waves in a self-loop's phases at priority 0, after a
    // loop (dispatch rounds, latency-bound) at 1, so the issue arbiter
    // prefers them over the loops' throughput-bound VALU streams (a wave
    // starts at 0)
    if (shape == JIT_MACHINE) {
        e.line("#define MK_PRIO_LOOP() __builtin_amdgcn_s_setprio(0)");
        e.line("#define MK_PRIO_REST() __builtin_amdgcn_s_setprio(1)");
    }
    // the machine lane's dispatch value as an SGPR value GVN cannot equate
    // with the lane's superblock id (MK_SCALAR, chosen by emit_machine_lane;
    // machine modules only, so the stream modules' sources stay as they were)
    if (shape == JIT_MACHINE)
        e.line("MK_FN uint32_t mk_scalar(uint32_t u) { uint32_t r; __asm__(\"\" : \"=s\"(r) : \"0\"(u)); return r; }");
    // int 0/1 loop flags and the predicated bump (emit_self_loop, narrow
    // phase); inline asm so that LLVM does not turn them back into lane masks
    e.line("MK_FN int32_t mk_flag_gt(int32_t x) { int32_t f; __asm__(\"v_med3_i32 %%0, %%1, 0, 1\" : \"=v\"(f) : \"v\"(x)); return f; }");
    e.line("MK_FN int32_t mk_flag_lt(int32_t x) { int32_t f; __asm__(\"v_lshrrev_b32 %%0, 31, %%1\" : \"=v\"(f) : \"v\"(x)); return f; }");
    e.line("MK_FN int32_t mk_flag_nz(int32_t x) { int32_t f; __asm__(\"v_min_u32 %%0, 1, %%1\" : \"=v\"(f) : \"v\"(x)); return f; }");
    // (in plain C the min stays v_min_u32 and the s_nop the hazard recognizer
    // puts after inline asm goes away, yet C5 ran 236.7 us against 215-221:
    // r03f, so asm)
    e.line("MK_FN int32_t mk_flag_min(int32_t x, int32_t g) { int32_t f; __asm__(\"v_min_u32 %%0, %%1, %%2\" : \"=v\"(f) : \"v\"(x), \"v\"(g)); return f; }");
    e.line("MK_FN int32_t mk_mad24(int32_t f, int32_t k, int32_t x)");
    e.line("{");
    e.line("    int32_t r;");
    e.line("    __asm__(\"v_mad_i32_i24 %%0, %%1, %%2, %%3\" : \"=v\"(r) : \"v\"(f), \"v\"(k), \"v\"(x));");
    e.line("    return r;");
    e.line("}");
    e.line("#define MK_FLAG_GT(x) mk_flag_gt(x)");
    e.line("#define MK_FLAG_LT(x) mk_flag_lt(x)");
    e.line("#define MK_FLAG_NZ(x) mk_flag_nz(x)");
    e.line("#define MK_FLAG_MIN(x, f) mk_flag_min((x), (f))");
    e.line("#define MK_MAD24(f, k, x) mk_mad24((f), (k), (x))");
    // the saturating countdown forms (emit_self_loop), only in modules that
    // use them (other modules' source -- and its hash -- stays as it was)
    if (sat) {
        // x - 1 saturating at 0 as unsigned (asm: LLVM folds a chain of them into one subtract)
        e.line("MK_FN int32_t mk_satdec(int32_t x) { int32_t r; __asm__(\"v_sub_u32_e64 %%0, %%1, 1 clamp\" : \"=v\"(r) : \"v\"(x)); return r; }");
        e.line("#define MK_SATDEC(x) mk_satdec(x)");
        // sat_block of them in one asm statement: the hazard recognizer's
        // s_nop after an asm statement then comes once per block
        // (MK_JIT_SAT_BLOCK)
        std::string b = "MK_FN int32_t mk_satdecb(int32_t x) { __asm__(\"";
        for (uint32_t k = 0; k < lim.sat_block; ++k) b += k ? "\\n\\tv_sub_u32_e64 %0, %0, 1 clamp" : "v_sub_u32_e64 %0, %0, 1 clamp";
        b += "\" : \"+v\"(x)); return x; }\n";
        e.s += b;
        e.line("#define MK_SATDECB(x) mk_satdecb(x)");
    }
    // stack-slot accesses
    e.line("#define MK_SLOT_ST(b, ss, s, v) ((b)[(uint64_t)(s) * (ss)] = (v))");
    e.line("#define MK_SLOT_LD(b, ss, s) ((b)[(uint64_t)(s) * (ss)])");
    // per-lane slot numbers (dynamic stacks); the buffer-op form redefines them.
    // Machine kernels (narrow_slots): slot x stride in one full-rate 24-bit
    // multiply (v_mul_u32_u24) instead of a 64 x 64-bit product (two
    // v_mad_u64_u32 and moves per access); the executor keeps stride < 2^24
    // and slots x stride < 2^32 (launch_jit_locked).
    if (narrow_slots) {
        e.line("extern \"C\" __device__ uint32_t __ockl_mul24_u32(uint32_t, uint32_t);");
        e.line("#define MK_SLOT_STX(b, ss, s, v) ((b)[__ockl_mul24_u32((uint32_t)(s), (uint32_t)(ss))] = (v))");
        e.line("#define MK_SLOT_LDX(b, ss, s) ((b)[__ockl_mul24_u32((uint32_t)(s), (uint32_t)(ss))])");
    } else {
        e.line("#define MK_SLOT_STX(b, ss, s, v) MK_SLOT_ST(b, ss, s, v)");
        e.line("#define MK_SLOT_LDX(b, ss, s) MK_SLOT_LD(b, ss, s)");
    }
    // vector out/status stores of the light stream kernel
    e.line("typedef int32_t mk_i32x4 __attribute__((ext_vector_type(4)));");
    e.line("#define MK_IO_ST(ptr, v) (*(ptr) = (v))");
    // loop policy of the machine shape (see kMachineKernel)
    e.line("MK_FN uint32_t mk_loop_need(uint32_t pol)");
    e.line("{");
    e.line("    const uint32_t g0 = (uint32_t)__popcll(__ballot(1));");
    e.line("    return g0 >= ((pol >> 16) & 0xffu) ? (g0 * ((pol >> 8) & 0xffu) + 15u) / 16u : 0u;");
    e.line("}");
    // wave-uniform: some lane of the group is still in the loop, and at least `need`
    e.line("MK_FN bool mk_keep(bool m, uint32_t need)");
    e.line("{");
    e.line("    const uint32_t c = (uint32_t)__popcll(__ballot(m));");
    e.line("    return c != 0u && c >= need;");
    e.line("}");
    e.line("#define MK_LOOP_NEED(pol) mk_loop_need(pol)");
    // max over the wave (ockl's DPP reduction: needs the whole wave active), as a scalar
    e.line("extern \"C\" __device__ uint32_t __ockl_wfred_max_u32(uint32_t);");
    e.line("#define MK_WAVE_MAX(x) __builtin_amdgcn_readfirstlane(__ockl_wfred_max_u32((uint32_t)(x)))");
    e.line("extern \"C\" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);");
    e.line("extern \"C\" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);");
    e.line("#define MK_WAVE_MIN(x) __builtin_amdgcn_readfirstlane(__ockl_wfred_min_u32((uint32_t)(x)))");
    e.line("#define MK_KEEP(m, need) mk_keep(m, need)");
    e.s += kDeviceCommon;
    e.s += "\n";
    return e.s;
}

// Stateful sessions (row f2): every thread one session instance, its lane
// state (superblock to start the next call at, registers, stack slots)
// loaded from and stored back to HBM; each of the launch's ncalls /compute
// calls runs the session schedule's superblocks by generations (the
// dispatcher of kMachineKernel) until the call yields.  A call whose budget
// slice would end inside a superblock hands off (MK_SS_HANDOFF): the lane
// stops at that superblock's entry, records it, and the interpreter
// (mk_exec.hip tis_session, which imports it first) finishes that call and the
// rest of the burst.  Sessions the interpreter holds (MK_SS_T1) are skipped.
const char *const kSessionKernel = R"(
struct SessK {
    uint64_t n;
    uint32_t ncalls, budget;
    const int64_t *in;   // [ncalls][n]
    int32_t *out;        // [ncalls][n]
    uint8_t *status;     // [ncalls][n]
    uint32_t *steps;     // [ncalls][n] or null
    uint32_t *sb;        // [n] variant the next call starts at, or MK_SS_*
    int64_t *regs;       // [register][n]
    int32_t *slots;      // [slot][n]
    uint32_t *hand_sb;   // [n] superblock of a hand-off
    uint32_t *hand_steps;// [n] the call's steps at it
    uint32_t *hand_call; // [n] the call of the burst it happened in
    uint32_t *sflags;    // [0]: this launch's epoch once a lane handed off (mk_exec.hip SessParams)
    uint32_t epoch;
};
extern "C" __global__ void __launch_bounds__(256) mk_sess_exec(SessK p)
{
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const bool live = gid < p.n;
    uint32_t sbv = live ? p.sb[gid] : MK_SS_DEAD;
    const bool native = sbv < MK_SS_DEAD;
    MkLane L;
    mk_sess_load(L, p.regs, gid, p.n, native);
    int32_t *slots = p.slots ? p.slots + gid : (int32_t *)0;
    for (uint32_t call = 0; call < p.ncalls; ++call) {
        const uint64_t ci = (uint64_t)call * p.n + gid;
        const bool run = sbv < MK_SS_DEAD;
        L.sb = run ? sbv : MK_SB_IDLE;
        L.steps = 0u;
        L.st = 0u;
        L.outv = 0;
        L.next = MK_SS_DEAD;
        if (run) mk_sess_input(L, (int64_t)(int32_t)p.in[ci]); // int32(v) at GetInput (master.go:237)
#if defined(MK_SWEEP_LIST)
        // sweep dispatch, as kMachineSortKernel's (JitLimits::sweep)
#define MK_SWEEP_STEP(v, loop)                                                                   \
        if (__ballot(L.sb == (v))) {                                                                 \
            const uint32_t smax_ = (loop) ? MK_WAVE_MAX(L.sb == (v) ? L.steps : 0u) : 0u;            \
            if (L.sb == (v)) mk_run((v), L, p.budget, slots, p.n, MK_POLICY, smax_);                 \
        }
        for (uint32_t ps = 0; ps < MK_SWEEP_PASSES && __ballot(L.sb < MK_SB_DONE); ++ps) {
            MK_SWEEP_LIST(MK_SWEEP_STEP)
#if defined(MK_SWEEP_COLD)
            if (__ballot(L.sb < 64u && ((MK_SWEEP_COLD_MASK >> L.sb) & 1ull))) {
                MK_SWEEP_COLD(MK_SWEEP_STEP)
            }
#endif
        }
#undef MK_SWEEP_STEP
#endif
        for (;;) { // rounds, for the lanes the sweep passes left
            const unsigned long long actb = __ballot(L.sb < MK_SB_DONE);
            if (!actb) break;
            const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)L.sb, (int)__builtin_ctzll(actb));
            const uint32_t smax = mk_is_loop(u) ? MK_WAVE_MAX(L.sb == u ? L.steps : 0u) : 0u;
            const uint32_t us = MK_SCALAR(u); // the switch value, out of GVN's reach (MK_JIT_UNIFORM_SW)
            if (L.sb == u) mk_run(us, L, p.budget, slots, p.n, MK_POLICY, smax);
        }
        if (!live || sbv == MK_SS_T1 || sbv == MK_SS_HAND) continue; // the interpreter answers these
        if (run && L.st == MK_SS_HANDOFF) {
            p.hand_sb[gid] = L.next / 2u;
            p.hand_steps[gid] = L.steps;
            p.hand_call[gid] = call;
            p.sflags[0] = p.epoch; // the import kernel has work
            sbv = MK_SS_HAND;
            continue;
        }
        p.out[ci] = run && (L.st & MK_ST_HAS_OUTPUT) ? L.outv : 0;
        p.status[ci] = (uint8_t)(run ? L.st : MK_ST_STACK_OVERFLOW);
        if (p.steps) p.steps[ci] = run ? L.steps : 0u;
        if (run) sbv = L.next;
    }
    if (native) {
        mk_sess_store(L, p.regs, gid, p.n);
        p.sb[gid] = sbv;
    }
}
)";
} // namespace

std::string jit_module_source(const std::string &lane_src, JitShape shape, bool heavy, const JitLimits &lim,
                              uint32_t pool)
{
    Emitter e;
    e.s = module_prelude(shape, lim, pool, lane_src.find("MK_SAT") != std::string::npos, shape == JIT_MACHINE);
    e.s += lane_src;
    const char *mk = lim.tile_sort && !lim.order ? kMachineSortKernel
                                                 : kMachineKernel;
    if (shape == JIT_MACHINE && pool >= 64) mk = kMachinePoolKernel;
    else if (shape == JIT_MACHINE && pool >= 2) mk = kMachineMultiKernel;
    if (shape != JIT_MACHINE) e.s += kStreamCount;
    e.s += shape == JIT_MACHINE ? mk : heavy ? kStreamKernelHeavy : kStreamKernel;
    return e.s;
}

} // namespace mk

namespace mk {

bool jit_session_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why)
{
    if (!p.session) {
        why = "not a session schedule";
        return false;
    }
    Graph g;
    if (!analyze(p, lim, g, why)) return false;
    Emitter e;
    emit_machine_lane(p, g, e);
    src = module_prelude(JIT_MACHINE, lim, 0, e.s.find("MK_SAT") != std::string::npos) + e.s + kSessionKernel;
    return true;
}

// The most node-instructions one /compute call can retire on the session
// schedule's fast variants: the longest path from a call's entry (variant 0,
// or where a U_YIELD sends the next call) to the U_YIELD or U_END that ends
// it; UINT64_MAX when a call can loop (a cycle between yields) or the
// schedule does not analyze.  A launch whose budget exceeds it never fires a
// budget guard, so no call hands off to the interpreter (round 4).
uint64_t jit_session_max_call_steps(const SchedProgram &p, const JitLimits &lim)
{
    if (!p.session) return UINT64_MAX;
    Graph g;
    std::string why;
    if (!analyze(p, lim, g, why)) return UINT64_MAX;
    const size_t nv = g.entry.size();
    // successors through the fast variant's exits, with the steps retired on
    // the way to each; a call ends at U_YIELD / U_END (its steps in `fin`)
    auto exits = [&](uint32_t v, std::vector<std::pair<uint32_t, uint64_t>> &succ, uint64_t &fin,
                     uint32_t &next) -> bool {
        succ.clear();
        fin = 0;
        next = ~0u;
        for (size_t pc = g.entry[v];; ++pc) {
            const DOp &I = g.D[pc];
            switch (I.op) {
            case U_GUARD: continue; // not taken when the budget exceeds every path
            case U_BRX: succ.push_back({(uint32_t)I.imm, I.inc}); continue;
            case U_JUMP: succ.push_back({(uint32_t)I.imm, I.inc}); return true;
            case U_BR:
                succ.push_back({(uint32_t)(uint64_t)I.imm, I.inc});
                succ.push_back({(uint32_t)((uint64_t)I.imm >> 32), I.inc});
                return true;
            case U_JRO:
                for (uint64_t t = 0; t <= I.b; ++t) succ.push_back({p.jtab[(size_t)I.imm + t], I.inc});
                return true;
            case U_OVF: fin = std::max<uint64_t>(fin, I.inc); continue; // a full dynamic stack ends the session here
            case U_YIELD: fin = std::max<uint64_t>(fin, I.inc); next = (uint32_t)(uint64_t)I.imm; return true;
            case U_END: fin = std::max<uint64_t>(fin, I.inc); return true;
            case U_HANDOFF: return false; // (only in checked variants, which the fast paths do not reach)
            default:
                if (I.op > U_DATA_LAST && I.op != U_ROUND_END) return false; // unknown control: no bound
                continue;
            }
        }
    };
    std::vector<int64_t> memo(nv, -1);
    std::vector<uint8_t> state(nv, 0);
    std::vector<uint32_t> roots{0u};
    std::vector<std::pair<uint32_t, uint64_t>> succ;
    uint64_t fin = 0, best_all = 0;
    uint32_t next = 0;
    for (size_t r = 0; r < roots.size(); ++r) {
        std::vector<uint32_t> stack{roots[r]};
        while (!stack.empty()) {
            const uint32_t v = stack.back();
            if (v >= nv) return UINT64_MAX;
            if (state[v] == 0) {
                state[v] = 1;
                if (!exits(v, succ, fin, next)) return UINT64_MAX;
                if (next != ~0u && std::find(roots.begin(), roots.end(), next) == roots.end()) roots.push_back(next);
                for (const auto &w : succ) {
                    if (w.first >= nv) return UINT64_MAX;
                    if (state[w.first] == 1) return UINT64_MAX; // a cycle inside a call
                    if (state[w.first] == 0) stack.push_back(w.first);
                }
                continue;
            }
            stack.pop_back();
            if (state[v] == 2) continue;
            (void)exits(v, succ, fin, next);
            int64_t best = (int64_t)fin;
            for (const auto &w : succ) best = std::max<int64_t>(best, (int64_t)w.second + memo[w.first]);
            memo[v] = best;
            state[v] = 2;
        }
        best_all = std::max<uint64_t>(best_all, (uint64_t)memo[roots[r]]);
    }
    return best_all;
}

bool jit_session_lane(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why)
{
    if (!p.session) {
        why = "not a session schedule";
        return false;
    }
    Graph g;
    if (!analyze(p, lim, g, why)) return false;
    Emitter e;
    emit_machine_lane(p, g, e);
    src = e.s;
    return true;
}

} // namespace mk
