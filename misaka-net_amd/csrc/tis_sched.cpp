// tis_sched.cpp -- schedule compiler (see tis_sched.h).
//
// The symbolic executor below restates the same update() semantics as the
// GPU interpreter in mk_exec.hip (program.go:219-566, stack.go:95-155,
// master.go:233-249) over abstract values:
//   DEAD   value can never be read again (liveness) -- not part of the state
//   CONST  compile-time constant (int64; int32-range for 32-bit locations)
//   REG    lives in a per-lane 64-bit register r (read as sext32 if `tr`)
//   MEM    a stack entry stored in its lane-major HBM slot
// Control is concrete.  A superblock ends where control depends on data
// (conditional jump / JRO on a non-constant), at termination, or where the
// state at a round end was already compiled (loops merge there).  At every
// exit the live symbolic values are moved into fixed per-location "home"
// registers so that all paths into a state agree on where values are.
#include "tis_sched.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <unordered_set>

#include "../../include/mk.h"

namespace mk {
namespace {

constexpr uint8_t K_DEAD = 0, K_CONST = 1, K_REG = 2, K_MEM = 3;

struct Val {
    uint8_t kind = K_DEAD;
    bool tr = false;
    uint16_t r = 0;
    int64_t c = 0;
};

inline Val vconst(int64_t c) { Val v; v.kind = K_CONST; v.c = c; return v; }
inline Val vdead() { return Val(); }
inline int64_t sext32(int64_t v) { return (int64_t)(int32_t)(uint32_t)(uint64_t)v; }
inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

inline uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Ctl {
    std::vector<uint16_t> ip;
    uint32_t pend = 0, hung = 0;
    uint64_t pfull = 0;
    std::vector<uint32_t> depth; // entries tracked symbolically (dynamic stacks: above the memory part)
    std::vector<uint8_t> lo;     // dynamic stacks: known lower bound of the memory depth (0 or 1)
    bool in_avail = true;
    uint8_t out_cnt = 0; // sessions: outChan full (0/1)
    uint8_t pos = 0;
    bool changed = false;
    // sessions: the call's input is deposited into inChan; the call's
    // round-start checks (deposit, take) are still to run at this state
    bool cdep = false, pre = false;
};

struct StackDigest {
    uint64_t h1 = 0, h2 = 0;
};

inline void digest_entry(StackDigest &g, uint32_t d, const Val &v, bool add)
{
    const uint64_t k = (v.kind == K_CONST) ? (uint64_t)v.c : 0x5359'4D42'4F4C'4943ull; // "SYMBOLIC"
    const uint64_t a = mix64(((uint64_t)d << 2) ^ (v.kind == K_CONST ? 1 : 2) ^ mix64(k));
    const uint64_t b = mix64(a ^ 0xA5A5'5A5A'C3C3'3C3Cull);
    if (add) { g.h1 += a; g.h2 += b; }
    else { g.h1 -= a; g.h2 -= b; }
}

struct EntryState {
    Ctl ctl;
    std::vector<Val> loc;               // K_DEAD / K_CONST / K_REG(home) -- REG means "in home"
    std::vector<std::vector<Val>> stk;  // K_CONST / K_MEM
    std::vector<StackDigest> dig;
};

enum { A_CONT = 0, A_EXIT = 1 };

class Compiler {
  public:
    Compiler(const Network &net, uint32_t cap, bool soo, const SchedLimits &lim, const std::vector<uint8_t> &dyn,
             bool sess = false)
        : net_(net), cap_(cap), soo_(soo), sess_(sess), lim_(lim), N_(net.nprog), S_(net.uses_stacks ? net.nstack : 0)
    {
        L0_ = 7 * N_ + 2 + S_ + (sess ? 1 : 0);
        home_.assign(L0_, -1);
        dyn_base_.assign(S_, -1);
        for (int s = 0; s < S_; s++)
            if ((size_t)s < dyn.size() && dyn[s]) dyn_base_[s] = (int64_t)(ndyn_++) * cap_;
        depths_seen_.assign(S_, {});
        want_dyn_.assign(S_, 0);
    }

    bool run(SchedProgram &out, std::string &why);
    // stacks whose depth should follow the data (set when the compile failed)
    const std::vector<uint8_t> &want_dyn() const { return want_dyn_; }

  private:
    // ---- location space -------------------------------------------------
    int ACC(int n) const { return n; }
    int BAK(int n) const { return N_ + n; }
    int PORT(int slot) const { return 2 * N_ + slot; }
    int PENDV(int n) const { return 6 * N_ + n; }
    int INL() const { return 7 * N_; }
    int OUTL() const { return 7 * N_ + 1; }
    int DEP(int s) const { return 7 * N_ + 2 + s; } // dynamic stack: entries in memory
    int CIN() const { return 7 * N_ + 2 + S_; }     // sessions: the call's input, not yet deposited
    bool is32(int loc) const { return (loc >= 2 * N_ && loc < 7 * N_ + 2) || (sess_ && loc == CIN()); }

    const Network &net_;
    uint32_t cap_;
    bool soo_;
    bool sess_; // stateful sessions: calls, inChan / outChan as channels (session_step)
    SchedLimits lim_;
    int N_, S_, L0_;
    std::vector<std::vector<uint8_t>> acc_live_, bak_live_;

    // homes (global, permanent)
    std::vector<int> home_;
    std::vector<uint8_t> claimed_; // register is some location's home

    // entries / work list
    std::vector<EntryState> entries_;
    std::unordered_map<std::string, uint32_t> memo_;
    std::deque<uint32_t> work_;
    std::vector<std::vector<UOp>> sb_code_; // per entry, with ROUND_END markers
    std::vector<uint32_t> jtab_;
    uint32_t total_words_ = 0;
    uint64_t rounds_ = 0;
    bool fail_ = false;
    std::string why_;

    // trace state
    Ctl ctl_;
    std::vector<Val> loc_;
    std::vector<std::vector<Val>> stk_;
    std::vector<StackDigest> dig_;
    std::vector<int> refcnt_;
    std::vector<uint8_t> r32_;
    std::vector<UOp> code_;
    uint32_t steps_ = 0;
    uint32_t max_reg_ = 0;
    uint32_t max_slot_ = 0;
    bool any_slot_ = false;
    std::vector<std::vector<int32_t>> slot_id_; // [stack][depth] -> dense HBM slot, -1 = none yet

    // Dynamic stacks.  A stack whose depth follows the data (a PUSH loop over
    // an input-dependent count) would make the control state -- depths are
    // part of it -- grow with the data.  Such a stack keeps its entries in a
    // contiguous slot range [base, base + cap) instead: the depth of its
    // memory part is a location (DEP: a constant 0, or a per-lane register),
    // and only the entries pushed since the last superblock exit are tracked
    // symbolically above it (ctl.depth = their number).  Every exit flushes
    // them (STX at base + DEP + j, DEP += n).  PUSH checks the capacity in
    // line (OVF); POP from an empty tracked part reads slot base + DEP - 1
    // (LDX) once DEP >= 1 is known, which a branch on DEP == 0 establishes
    // (taken: the stack is empty -- DEP becomes the constant 0 and the POP
    // blocks; not taken: lo = 1).
    std::vector<int64_t> dyn_base_; // first slot of a dynamic stack, -1 = ordinary stack
    uint32_t ndyn_ = 0;
    std::vector<std::unordered_set<uint32_t>> depths_seen_; // ordinary stacks: depths at superblock entries
    std::vector<uint8_t> want_dyn_;

    bool dyn(int s) const { return dyn_base_[s] >= 0; }

    uint32_t slot_of(int s, uint32_t d)
    {
        any_slot_ = true;
        if (dyn(s)) return (uint32_t)(dyn_base_[s] + d);
        if (slot_id_.size() < (size_t)S_) slot_id_.resize(S_);
        auto &v = slot_id_[s];
        if (v.size() <= d) v.resize(d + 1, -1);
        if (v[d] < 0) v[d] = (int32_t)max_slot_++;
        return (uint32_t)(ndyn_ * cap_ + v[d]);
    }

    // ---- helpers --------------------------------------------------------
    void failf(const std::string &w)
    {
        if (!fail_) { fail_ = true; why_ = w; }
    }
    void ensure_reg(int r)
    {
        if ((size_t)r >= refcnt_.size()) {
            refcnt_.resize(r + 1, 0);
            r32_.resize(r + 1, 0);
            claimed_.resize(r + 1, 0);
        }
        if ((uint32_t)r + 1 > max_reg_) max_reg_ = r + 1;
        if ((uint32_t)r >= lim_.max_regs) failf("register budget exceeded");
    }
    void incref(const Val &v)
    {
        if (v.kind == K_REG) { ensure_reg(v.r); refcnt_[v.r]++; }
    }
    void decref(const Val &v)
    {
        if (v.kind == K_REG) refcnt_[v.r]--;
    }
    void set_loc(int X, Val v)
    {
        incref(v);
        decref(loc_[X]);
        loc_[X] = v;
    }
    // a value as stored into a 32-bit location (int32() at every hop)
    Val trunc(const Val &v)
    {
        if (v.kind == K_CONST) return vconst(sext32(v.c));
        if (v.kind == K_REG) {
            Val w = v;
            w.tr = !r32_[v.r];
            return w;
        }
        return v;
    }
    int fresh_reg(const std::vector<uint8_t> *exclude = nullptr)
    {
        for (;;) {
            int r = 0;
            for (;; r++) {
                if ((size_t)r >= refcnt_.size() || (refcnt_[r] == 0 && !(exclude && (size_t)r < exclude->size() && (*exclude)[r])))
                    break;
            }
            if ((uint32_t)r < lim_.soft_regs || !spill_one()) {
                ensure_reg(r);
                return r;
            }
        }
    }
    // Store the oldest register-only stack entry to its HBM slot.
    bool spill_one()
    {
        for (uint32_t d = 0;; d++) {
            bool any = false;
            for (int s = 0; s < S_; s++) {
                if (d >= stk_[s].size()) continue;
                any = true;
                Val &v = stk_[s][d];
                if (v.kind == K_REG && refcnt_[v.r] == 1) {
                    st_entry(s, d, v);
                    decref(v);
                    v = Val();
                    v.kind = K_MEM; // digest unchanged: still symbolic
                    return true;
                }
            }
            if (!any) return false;
        }
    }
    void emit(uint8_t op, uint8_t fl, uint32_t d, uint32_t a, uint32_t b, int64_t imm)
    {
        UOp u;
        u.op = op;
        u.fl = fl;
        u.d = (uint16_t)d;
        u.a = (uint16_t)a;
        u.b = (uint16_t)b;
        u.imm = imm;
        code_.push_back(u);
    }
    void emit_ext(int64_t imm) { emit(0xFF, 0, 0, 0, 0, imm); }

    // Store tracked entry d of stack s (value v: CONST or REG) to its slot:
    // static for ordinary stacks and over a constant DEP, indexed by the DEP
    // register otherwise.  Never allocates for a REG value (spill_one calls it).
    void st_entry(int s, uint32_t d, const Val &v)
    {
        const Val &D = dyn(s) ? loc_[DEP(s)] : Val();
        if (!dyn(s) || D.kind == K_CONST) {
            const uint32_t slot = slot_of(s, (uint32_t)(dyn(s) ? D.c : 0) + d);
            if (v.kind == K_CONST) emit(U_STI, 0, 0, slot & 0xFFFF, slot >> 16, v.c);
            else emit(U_ST, fa(v), 0, v.r, 0, slot);
            return;
        }
        any_slot_ = true;
        int src = v.r;
        uint8_t fl = fa(v);
        if (v.kind == K_CONST) {
            src = fresh_reg();
            emit(U_LI, 0, src, 0, 0, v.c);
            fl = 0;
        }
        emit(U_STX, fl, 0, src, D.r, dyn_base_[s] + d);
    }
    // Load tracked entry d (K_MEM) of stack s into register r.
    void ld_entry(int s, uint32_t d, int r)
    {
        const Val &D = dyn(s) ? loc_[DEP(s)] : Val();
        if (!dyn(s) || D.kind == K_CONST) {
            emit(U_LD, 0, r, 0, 0, slot_of(s, (uint32_t)(dyn(s) ? D.c : 0) + d));
            return;
        }
        any_slot_ = true;
        emit(U_LDX, 0, r, 0, D.r, dyn_base_[s] + d);
    }
    // DEP(s) += k (dynamic stack), as a register.
    void dep_add(int s, int64_t k)
    {
        const Val D = loc_[DEP(s)];
        const int d = dest_for(DEP(s));
        if (D.kind == K_CONST) emit(U_LI, 0, d, 0, 0, D.c + k);
        else emit(U_ADDI, 0, d, D.r, 0, k);
        Val nv;
        nv.kind = K_REG;
        nv.r = (uint16_t)d;
        set_loc(DEP(s), nv);
        r32_[d] = 0;
    }
    // At a superblock exit: every dynamic stack's tracked entries go to memory.
    void flush_dyn()
    {
        for (int s = 0; s < S_; s++) {
            if (!dyn(s) || stk_[s].empty()) continue;
            const uint32_t n = (uint32_t)stk_[s].size();
            for (uint32_t d = 0; d < n; d++) {
                Val &v = stk_[s][d];
                if (v.kind == K_CONST || v.kind == K_REG) st_entry(s, d, v);
                decref(v);
                v = Val();
            }
            const Val D = loc_[DEP(s)];
            const int64_t lo = D.kind == K_CONST ? D.c + n : (int64_t)ctl_.lo[s] + n;
            dep_add(s, n);
            stk_[s].clear();
            dig_[s] = StackDigest();
            ctl_.depth[s] = 0;
            ctl_.lo[s] = (uint8_t)std::min<int64_t>(lo, 1);
        }
    }
    uint8_t fa(const Val &v) const { return v.tr ? UF_TA : 0; }
    uint8_t fb(const Val &v) const { return v.tr ? UF_TB : 0; }

    // destination register for a new value of location X
    int dest_for(int X)
    {
        const Val &cur = loc_[X];
        if (cur.kind == K_REG && refcnt_[cur.r] == 1) return cur.r;
        return fresh_reg();
    }

    void op_addsub(int X, Val a, Val b, bool sub)
    {
        if (a.kind == K_CONST && b.kind == K_CONST) {
            set_loc(X, vconst(sub ? wsub(a.c, b.c) : wadd(a.c, b.c)));
            return;
        }
        // sources are referenced by locations or by the attempt's hold, so
        // fresh_reg() cannot hand out their registers
        const int d = dest_for(X);
        if (b.kind == K_CONST)
            emit(U_ADDI, fa(a), d, a.r, 0, sub ? wsub(0, b.c) : b.c);
        else if (a.kind == K_CONST) {
            if (sub) emit(U_RSUBI, fa(b), d, b.r, 0, a.c);
            else emit(U_ADDI, fa(b), d, b.r, 0, a.c);
        } else {
            emit(sub ? U_SUB : U_ADD, (uint8_t)(fa(a) | fb(b)), d, a.r, b.r, 0);
        }
        Val nv;
        nv.kind = K_REG;
        nv.r = (uint16_t)d;
        set_loc(X, nv);
        r32_[d] = 0;
    }

    // ---- liveness of ACC / BAK per node instruction ----------------------
    void liveness();
    // ---- stacks whose memory slots are never in use together share them --
    void share_slots();

    // ---- state management ---------------------------------------------
    void prune(Ctl &c, std::vector<Val> &loc) const;
    std::string key_of(const Ctl &c, const std::vector<Val> &loc, const std::vector<StackDigest> &dig) const;
    std::string shape_of(const Ctl &c, const std::vector<Val> &loc, const std::vector<StackDigest> &dig) const;
    std::unordered_map<std::string, uint32_t> shape_count_;
    uint32_t get_or_create(const Ctl &c, const std::vector<Val> &loc);
    void load_entry(uint32_t id);

    // ---- exits ----------------------------------------------------------
    // Moves every location that is symbolic in any successor into its home
    // register and stores symbolic stack entries.  `keep` is a value the
    // exit op still reads afterwards; returns where to read it.
    Val canonicalize(std::vector<Ctl> &succ, std::vector<std::vector<Val>> &succ_loc, Val keep,
                     std::vector<uint8_t> *need_out = nullptr);
    void rehome(const std::vector<uint8_t> &need);
    void exit_jump();
    void exit_end(uint8_t reason);
    void exit_branch(int n, uint8_t cond, uint16_t target);
    void exit_jro(int n, const Val &v);
    bool inline_pop_check(int s);
    void round_end_marker();
    void generalize();
    // sessions
    void exit_yield(uint8_t reason);
    bool session_round_start();
    uint8_t out_bit() const { return !sess_ && ctl_.out_cnt > 0 ? MK_ST_HAS_OUTPUT : 0; }
    Val out_val() const { return sess_ ? vconst(0) : loc_[OUTL()]; }

    int attempt(int n);
    void compile_entry(uint32_t id);
};

void Compiler::liveness()
{
    acc_live_.assign(N_, {});
    bak_live_.assign(N_, {});
    for (int n = 0; n < N_; n++) {
        const uint32_t len = net_.len[n];
        const Insn *code = &net_.code[net_.base[n]];
        std::vector<uint8_t> al(len, 0), bl(len, 0);
        bool changed = true;
        while (changed) {
            changed = false;
            for (int64_t i = (int64_t)len - 1; i >= 0; i--) {
                const Insn &I = code[i];
                bool ao = false, bo = false;
                auto succ = [&](int64_t t) {
                    ao = ao || al[t];
                    bo = bo || bl[t];
                };
                const int64_t nx = (i + 1 == (int64_t)len) ? 0 : i + 1;
                switch (I.op) {
                case OP_JMP: succ(I.arg); break;
                case OP_JEZ: case OP_JNZ: case OP_JGZ: case OP_JLZ: succ(I.arg); succ(nx); break;
                case OP_JRO:
                    if (I.src == SRC_IMM) {
                        int64_t t = wadd(i, I.imm);
                        t = std::min<int64_t>(std::max<int64_t>(t, 0), (int64_t)len - 1);
                        succ(t);
                    } else {
                        for (uint32_t t = 0; t < len; t++) succ(t);
                    }
                    break;
                case OP_STUCK: case OP_HANG: case OP_RETRY: break;
                default: succ(nx); break;
                }
                const bool src_acc = I.src == SRC_ACC;
                bool a = ao, b = bo;
                switch (I.op) {
                case OP_NOP: case OP_JMP: case OP_NEG: case OP_ADD: case OP_SUB: break;
                case OP_JEZ: case OP_JNZ: case OP_JGZ: case OP_JLZ: a = true; break;
                case OP_SWP: a = bo; b = ao; break;
                case OP_SAV: a = ao || bo; b = false; break;
                case OP_MOV: a = I.dst ? (src_acc && ao) : (ao || src_acc); break;
                case OP_JRO: case OP_SEND: case OP_PUSH: case OP_OUT: a = ao || src_acc; break;
                case OP_HANG: case OP_RETRY: a = src_acc; b = false; break;
                case OP_STUCK: a = false; b = false; break;
                case OP_POP: case OP_IN: if (I.dst) a = false; break;
                default: break;
                }
                if (a != (bool)al[i] || b != (bool)bl[i]) {
                    al[i] = a;
                    bl[i] = b;
                    changed = true;
                }
            }
        }
        acc_live_[n] = al;
        bak_live_[n] = bl;
    }
}

void Compiler::prune(Ctl &c, std::vector<Val> &loc) const
{
    for (int n = 0; n < N_; n++) {
        const bool h = (c.hung >> n) & 1u;
        if (h || !acc_live_[n][c.ip[n]]) loc[ACC(n)] = vdead();
        if (h || !bak_live_[n][c.ip[n]]) loc[BAK(n)] = vdead();
        if (!((c.pend >> n) & 1u)) loc[PENDV(n)] = vdead();
    }
    for (int s = 0; s < 4 * N_; s++)
        if (!((c.pfull >> s) & 1ull)) loc[PORT(s)] = vdead();
    if (!c.in_avail) loc[INL()] = vdead();
    if (sess_) {
        if (!c.out_cnt) loc[OUTL()] = vdead();
        if (c.cdep) loc[CIN()] = vdead();
    }
}

// key_of without the constants' values (what widening compares)
std::string Compiler::shape_of(const Ctl &c, const std::vector<Val> &loc, const std::vector<StackDigest> &dig) const
{
    std::vector<Val> l = loc;
    for (int X = 0; X < 7 * N_ + 2; X++)
        if (l[X].kind == K_CONST) l[X].c = 0;
    return key_of(c, l, dig);
}

std::string Compiler::key_of(const Ctl &c, const std::vector<Val> &loc, const std::vector<StackDigest> &dig) const
{
    std::string k;
    k.reserve(64 + 2 * N_ + 10 * L0_ + 16 * S_);
    auto put = [&](const void *p, size_t n) { k.append((const char *)p, n); };
    put(c.ip.data(), c.ip.size() * 2);
    put(&c.pend, 4);
    put(&c.hung, 4);
    put(&c.pfull, 8);
    put(c.depth.data(), c.depth.size() * 4);
    put(c.lo.data(), c.lo.size());
    const uint8_t misc[6] = {(uint8_t)c.in_avail, c.out_cnt, c.pos, (uint8_t)c.changed, (uint8_t)c.cdep,
                             (uint8_t)c.pre};
    put(misc, 6);
    for (int X = 0; X < L0_; X++) {
        const Val &v = loc[X];
        const uint8_t kd = v.kind == K_MEM ? K_REG : v.kind;
        k.push_back((char)kd);
        if (kd == K_CONST) put(&v.c, 8);
    }
    for (int s = 0; s < S_; s++) {
        put(&dig[s].h1, 8);
        put(&dig[s].h2, 8);
    }
    return k;
}

uint32_t Compiler::get_or_create(const Ctl &c, const std::vector<Val> &loc)
{
    const std::string k = key_of(c, loc, dig_);
    auto it = memo_.find(k);
    if (it != memo_.end()) return it->second;
    for (int s = 0; s < S_; s++) {
        if (dyn(s)) continue;
        auto &seen = depths_seen_[s];
        seen.insert(c.depth[s]);
        if (lim_.dyn_depths && seen.size() > lim_.dyn_depths) { // the depth follows the data
            want_dyn_[s] = 1;
            failf("stack depth follows the data");
        }
    }
    if (fail_) return 0;
    if (entries_.size() >= lim_.max_superblocks) {
        for (int s = 0; s < S_; s++)
            if (!dyn(s) && lim_.dyn_depths && depths_seen_[s].size() > 1) want_dyn_[s] = 1;
        failf("superblock budget exceeded");
        return 0;
    }
    EntryState e;
    e.ctl = c;
    e.loc.resize(L0_);
    for (int X = 0; X < L0_; X++) {
        const Val &v = loc[X];
        if (v.kind == K_REG || v.kind == K_MEM) {
            Val h;
            h.kind = K_REG;
            h.r = (uint16_t)home_[X];
            e.loc[X] = h;
        } else {
            e.loc[X] = v;
        }
    }
    e.stk.resize(S_);
    for (int s = 0; s < S_; s++) {
        e.stk[s].reserve(stk_[s].size());
        for (const Val &v : stk_[s]) {
            if (v.kind == K_CONST) e.stk[s].push_back(v);
            else { Val m; m.kind = K_MEM; e.stk[s].push_back(m); }
        }
    }
    e.dig = dig_;
    const uint32_t id = (uint32_t)entries_.size();
    if (lim_.widen_after) shape_count_[shape_of(c, loc, dig_)]++;
    entries_.push_back(std::move(e));
    memo_.emplace(k, id);
    work_.push_back(id);
    return id;
}

void Compiler::load_entry(uint32_t id)
{
    const EntryState &e = entries_[id];
    ctl_ = e.ctl;
    std::fill(refcnt_.begin(), refcnt_.end(), 0);
    std::fill(r32_.begin(), r32_.end(), 0);
    loc_ = e.loc;
    for (int X = 0; X < L0_; X++) {
        if (loc_[X].kind == K_REG) {
            ensure_reg(loc_[X].r);
            refcnt_[loc_[X].r]++;
            r32_[loc_[X].r] = is32(X);
        }
    }
    stk_ = e.stk;
    dig_ = e.dig;
    code_.clear();
    steps_ = 0;
}

Val Compiler::canonicalize(std::vector<Ctl> &succ, std::vector<std::vector<Val>> &succ_loc, Val keep,
                           std::vector<uint8_t> *need_out)
{
    // 0. dynamic stacks: tracked entries to memory
    for (int s = 0; s < S_; s++) {
        if (!dyn(s) || stk_[s].empty()) continue;
        flush_dyn();
        for (Ctl &c : succ)
            for (int t = 0; t < S_; t++)
                if (dyn(t) && c.depth[t] != ctl_.depth[t]) c.depth[t] = ctl_.depth[t], c.lo[t] = ctl_.lo[t];
        break;
    }
    // 1. which locations must be in their home (symbolic in any successor)
    std::vector<uint8_t> need(L0_, 0);
    succ_loc.assign(succ.size(), loc_);
    for (size_t i = 0; i < succ.size(); i++) {
        Ctl c = succ[i];
        prune(c, succ_loc[i]);
        // widening: a successor whose state differs from lim_.widen_after
        // compiled states only in constants (a counter that changes every
        // iteration of a loop on data) gets its constants as registers
        if (lim_.widen_after && shape_count_[shape_of(c, succ_loc[i], dig_)] >= lim_.widen_after) {
            for (int X = 0; X < 7 * N_ + 2; X++) {
                if (succ_loc[i][X].kind != K_CONST) continue;
                succ_loc[i][X].kind = K_REG;
                need[X] = 1;
            }
        }
        for (int X = 0; X < L0_; X++)
            if (succ_loc[i][X].kind == K_REG || succ_loc[i][X].kind == K_MEM) need[X] = 1;
    }
    // 2. stack entries: symbolic values go to their HBM slot
    for (int s = 0; s < S_; s++) {
        for (uint32_t d = 0; d < (uint32_t)stk_[s].size(); d++) {
            Val &v = stk_[s][d];
            if (v.kind == K_REG) {
                st_entry(s, d, v);
                decref(v);
                v = Val();
                v.kind = K_MEM;
            }
        }
    }
    // 3. homes
    for (int X = 0; X < L0_; X++) {
        if (!need[X] || home_[X] >= 0) continue;
        const Val &v = loc_[X];
        if (v.kind == K_REG && !v.tr && !claimed_[v.r]) {
            // adopt the register the value already lives in ...
            bool shared = false;
            for (int Y = 0; Y < L0_ && !shared; Y++)
                shared = Y != X && need[Y] && home_[Y] < 0 && loc_[Y].kind == K_REG && loc_[Y].r == v.r && Y < X;
            if (!shared) {
                home_[X] = v.r;
                claimed_[v.r] = 1;
                continue;
            }
        }
        // ... or take a register nobody claims and nothing currently uses
        for (int r = 0;; r++) {
            ensure_reg(r);
            if (fail_) return keep;
            if (!claimed_[r] && refcnt_[r] == 0) {
                home_[X] = r;
                claimed_[r] = 1;
                break;
            }
        }
    }
    // 4. parallel moves into homes
    struct Mv { int dst, src; bool tr; };
    std::vector<Mv> mv;
    std::vector<std::pair<int, int64_t>> lis; // constants into homes, after the moves
    std::vector<uint8_t> isdst;
    for (int X = 0; X < L0_; X++) {
        if (!need[X]) continue;
        const Val &v = loc_[X];
        const int h = home_[X];
        if (v.kind == K_CONST) {
            // constant in this trace but symbolic in a merged successor
            lis.push_back({h, v.c});
            continue;
        }
        if (v.kind != K_REG) continue;
        if (v.r == h && !v.tr) continue;
        mv.push_back({h, v.r, v.tr});
    }
    isdst.assign(refcnt_.size() + 1, 0);
    for (auto &m : mv) {
        ensure_reg(m.dst);
        if ((size_t)m.dst >= isdst.size()) isdst.resize(m.dst + 1, 0);
        isdst[m.dst] = 1;
    }
    for (auto &l : lis) {
        ensure_reg(l.first);
        if ((size_t)l.first >= isdst.size()) isdst.resize(l.first + 1, 0);
        isdst[l.first] = 1;
    }
    // preserve `keep` if a move or a constant overwrites its register
    if (keep.kind == K_REG) {
        bool clobbered = false;
        for (auto &m : mv)
            if (m.dst == keep.r && !(m.src == keep.r && m.tr && keep.tr)) clobbered = true;
        for (auto &l : lis)
            if (l.first == keep.r) clobbered = true;
        if (clobbered) {
            std::vector<uint8_t> ex = isdst;
            for (auto &m : mv) {
                if ((size_t)m.src >= ex.size()) ex.resize(m.src + 1, 0);
                ex[m.src] = 1;
            }
            const int t = fresh_reg(&ex);
            emit(U_MOV, fa(keep), t, keep.r, 0, 0);
            keep.r = (uint16_t)t;
            keep.tr = false;
        }
    }
    while (!mv.empty()) {
        bool progress = false;
        for (size_t i = 0; i < mv.size(); i++) {
            bool read = false;
            for (size_t j = 0; j < mv.size() && !read; j++)
                read = j != i && mv[j].src == mv[i].dst;
            if (!read) {
                emit(U_MOV, mv[i].tr ? UF_TA : 0, mv[i].dst, mv[i].src, 0, 0);
                mv.erase(mv.begin() + i);
                progress = true;
                break;
            }
        }
        if (progress) continue;
        // only cycles left: park one destination's current content in a temp
        const int d = mv[0].dst;
        // not a register a move already wrote (a home whose new value is in
        // place) nor a pending destination, source or the exit's operand
        std::vector<uint8_t> ex = isdst;
        if (ex.size() < refcnt_.size() + 1) ex.resize(refcnt_.size() + 1, 0);
        for (auto &m : mv) {
            if ((size_t)std::max(m.dst, m.src) >= ex.size()) ex.resize(std::max(m.dst, m.src) + 1, 0);
            ex[m.dst] = ex[m.src] = 1;
        }
        if (keep.kind == K_REG) { // the exit op still reads it (it may sit in a temp of its own)
            if ((size_t)keep.r >= ex.size()) ex.resize(keep.r + 1, 0);
            ex[keep.r] = 1;
        }
        const int t = fresh_reg(&ex);
        if (fail_) return keep;
        emit(U_MOV, 0, t, d, 0, 0);
        for (auto &m : mv)
            if (m.src == d) m.src = t;
    }
    for (auto &l : lis) emit(U_LI, 0, l.first, 0, 0, l.second);
    if (keep.kind == K_REG) ensure_reg(keep.r);
    if (need_out) *need_out = need;
    return keep;
}

void Compiler::exit_jump()
{
    std::vector<Ctl> succ{ctl_};
    std::vector<std::vector<Val>> sl;
    canonicalize(succ, sl, Val());
    if (fail_) return;
    const uint32_t id = get_or_create(succ[0], sl[0]);
    emit(U_JUMP, 0, steps_ & 0xFFFF, steps_ >> 16, 0, 2 * (int64_t)id);
}

void Compiler::exit_end(uint8_t reason)
{
    const Val o = out_val();
    const uint8_t st = reason | out_bit();
    if (o.kind == K_REG) emit(U_END, (uint8_t)(UF_OUTREG | fa(o)), st, o.r, 0, 0);
    else emit(U_END, 0, st, 0, 0, o.kind == K_CONST ? o.c : 0);
    emit_ext(steps_);
}

void Compiler::exit_branch(int n, uint8_t cond, uint16_t target)
{
    const uint32_t len = net_.len[n];
    Ctl t = ctl_, f = ctl_;
    t.ip[n] = target;
    f.ip[n] = (uint16_t)(((uint32_t)ctl_.ip[n] + 1 == len) ? 0 : ctl_.ip[n] + 1);
    t.changed = f.changed = true;
    t.pos = f.pos = (uint8_t)(n + 1);
    steps_++;
    std::vector<Ctl> succ{t, f};
    std::vector<std::vector<Val>> sl;
    const Val a = canonicalize(succ, sl, loc_[ACC(n)]);
    if (fail_) return;
    const uint32_t it = get_or_create(succ[0], sl[0]);
    const uint32_t iff = get_or_create(succ[1], sl[1]);
    const int64_t imm = (int64_t)(((uint64_t)(2 * iff) << 32) | (uint64_t)(2 * it));
    emit(U_BR, (uint8_t)(fa(a) | (cond << UF_COND_SHIFT)), 0, a.r, 0, imm);
    emit_ext(steps_);
}

void Compiler::exit_jro(int n, const Val &v)
{
    const uint32_t len = net_.len[n];
    std::vector<Ctl> succ(len, ctl_);
    for (uint32_t t = 0; t < len; t++) {
        succ[t].ip[n] = (uint16_t)t;
        succ[t].changed = true;
        succ[t].pos = (uint8_t)(n + 1);
    }
    steps_++;
    std::vector<std::vector<Val>> sl;
    const Val a = canonicalize(succ, sl, v);
    if (fail_) return;
    const uint32_t off = (uint32_t)jtab_.size();
    jtab_.resize(off + len);
    for (uint32_t t = 0; t < len; t++) {
        const uint32_t id = get_or_create(succ[t], sl[t]);
        if (fail_) return;
        jtab_[off + t] = 2 * id;
    }
    emit(U_JRO, fa(a), ctl_.ip[n], a.r, (uint16_t)(len - 1), off);
    emit_ext(steps_);
}

// After a canonicalize() whose trace goes on (an in-line side exit): the
// values the successors need are in their homes, the others are dead.
void Compiler::rehome(const std::vector<uint8_t> &need)
{
    for (int X = 0; X < L0_; X++) {
        Val &v = loc_[X];
        if (v.kind != K_REG && v.kind != K_MEM) continue;
        if (need[X]) {
            v = Val();
            v.kind = K_REG;
            v.r = (uint16_t)home_[X];
        } else {
            v = vdead();
        }
    }
    std::fill(refcnt_.begin(), refcnt_.end(), 0);
    for (int X = 0; X < L0_; X++) {
        incref(loc_[X]);
        if (loc_[X].kind == K_REG) r32_[loc_[X].r] = is32(X);
    }
    for (int s = 0; s < S_; s++)
        for (const Val &e : stk_[s]) incref(e);
}

// POP from a dynamic stack whose memory part may be empty, in line: the
// lanes whose DEP is 0 leave through a side exit (BRX) to the state that
// knows the stack is empty (DEP the constant 0, the same node re-attempts
// the POP, which blocks); the others go on in this superblock knowing
// DEP >= 1.  Returns false when the exit could not be made (limits).
bool Compiler::inline_pop_check(int s)
{
    std::vector<Ctl> succ{ctl_};
    std::vector<std::vector<Val>> sl;
    std::vector<uint8_t> need;
    const Val a = canonicalize(succ, sl, loc_[DEP(s)], &need);
    if (fail_) return false;
    sl[0][DEP(s)] = vconst(0);
    const uint32_t it = get_or_create(succ[0], sl[0]);
    if (fail_) return false;
    emit(U_BRX, (uint8_t)(fa(a) | (0 << UF_COND_SHIFT)), 0, a.r, 0, 2 * (int64_t)it);
    emit_ext(steps_);
    rehome(need);
    ctl_.lo[s] = 1;
    return true;
}

void Compiler::round_end_marker()
{
    const Val o = out_val();
    const uint8_t st = MK_ST_BUDGET | out_bit();
    if (o.kind == K_REG) emit(U_ROUND_END, (uint8_t)(UF_OUTREG | fa(o)), st, o.r, 0, 0);
    else emit(U_ROUND_END, 0, st, 0, 0, o.kind == K_CONST ? o.c : 0);
    emit_ext(steps_);
}

// Sessions: a /compute call ends -- its output taken from outChan
// (MK_ST_HAS_OUTPUT) or a round without change (MK_ST_QUIESCENT: nothing can
// change without another input; the instance keeps its state).  The next
// call starts at the successor state with its input in CIN's home.
void Compiler::exit_yield(uint8_t reason)
{
    Ctl c = ctl_;
    c.pre = true;
    c.cdep = false;
    c.pos = 0;
    c.changed = false;
    Val o;
    if (reason & MK_ST_HAS_OUTPUT) {
        o = loc_[OUTL()];
        c.out_cnt = 0;
    }
    // the next call's input arrives in CIN's home (nothing else ever lives
    // there, so nothing moves), and the successor's shape must say so for
    // widening to see repeated states (a running sum across calls)
    Val in;
    in.kind = K_REG;
    in.r = (uint16_t)home_[CIN()];
    set_loc(CIN(), in);
    std::vector<Ctl> succ{c};
    std::vector<std::vector<Val>> sl;
    o = canonicalize(succ, sl, o);
    if (fail_) return;
    const uint32_t id = get_or_create(succ[0], sl[0]);
    if (fail_) return;
    const int64_t oc = o.kind == K_CONST ? sext32(o.c) : 0;
    if (o.kind == K_REG) emit(U_YIELD, (uint8_t)(UF_OUTREG | fa(o)), reason, o.r, 0, 2 * (int64_t)id);
    else emit(U_YIELD, 0, reason, 0, 0, 2 * (int64_t)id);
    emit_ext((int64_t)(((uint64_t)(uint32_t)oc << 32) | steps_));
}

// Sessions: the checks at the top of every round (tis_oracle.c
// session_step): the call's input goes into inChan once it is empty
// (m.inChan <- v, master.go:216); once deposited, a value in outChan ends
// the call (<-m.outChan, :219).  Returns true when the call ended.
bool Compiler::session_round_start()
{
    ctl_.pre = false;
    if (!ctl_.cdep && !ctl_.in_avail) {
        ctl_.in_avail = true;
        set_loc(INL(), loc_[CIN()]);
        set_loc(CIN(), vdead());
        ctl_.cdep = true;
    }
    if (ctl_.cdep && ctl_.out_cnt) {
        exit_yield(MK_ST_HAS_OUTPUT);
        return true;
    }
    return false;
}

void Compiler::generalize()
{
    // constants that keep changing (a loop over constant data) prevent the
    // state from ever repeating: turn every live constant into a register.
    for (int X = 0; X < 7 * N_ + 2; X++) { // not DEP: a constant DEP is 0 (empty)
        if (loc_[X].kind != K_CONST) continue;
        const int d = fresh_reg();
        emit(U_LI, 0, d, 0, 0, loc_[X].c);
        Val nv;
        nv.kind = K_REG;
        nv.r = (uint16_t)d;
        set_loc(X, nv);
        r32_[d] = is32(X);
    }
    for (int s = 0; s < S_; s++) {
        for (uint32_t d = 0; d < (uint32_t)stk_[s].size(); d++) {
            Val &v = stk_[s][d];
            if (v.kind != K_CONST) continue;
            st_entry(s, d, v);
            digest_entry(dig_[s], d, v, false);
            v = Val();
            v.kind = K_MEM;
            digest_entry(dig_[s], d, v, true);
        }
    }
}

int Compiler::attempt(int n)
{
    if ((ctl_.hung >> n) & 1u) return A_CONT;
    const uint32_t len = net_.len[n];
    uint16_t &ip = ctl_.ip[n];
    const Insn &I = net_.code[net_.base[n] + ip];
    auto retire = [&]() {
        ip = (uint16_t)(((uint32_t)ip + 1 == len) ? 0 : ip + 1);
        steps_++;
        ctl_.changed = true;
    };
    auto jump = [&](uint32_t t) {
        ip = (uint16_t)t;
        steps_++;
        ctl_.changed = true;
    };
    const int A = ACC(n);
    switch (I.op) {
    case OP_NOP: retire(); return A_CONT;
    case OP_SWP: std::swap(loc_[A], loc_[BAK(n)]); retire(); return A_CONT;
    case OP_SAV: set_loc(BAK(n), loc_[A]); retire(); return A_CONT;
    case OP_NEG: op_addsub(A, vconst(0), loc_[A], true); retire(); return A_CONT;
    case OP_JMP: jump(I.arg); return A_CONT;
    case OP_JEZ: case OP_JNZ: case OP_JGZ: case OP_JLZ: {
        const Val &a = loc_[A];
        if (a.kind == K_CONST) {
            const int64_t v = a.c;
            const bool take = (I.op == OP_JEZ && v == 0) || (I.op == OP_JNZ && v != 0) ||
                              (I.op == OP_JGZ && v > 0) || (I.op == OP_JLZ && v < 0);
            if (take) jump(I.arg);
            else retire();
            return A_CONT;
        }
        exit_branch(n, (uint8_t)(I.op - OP_JEZ), I.arg);
        return A_EXIT;
    }
    case OP_STUCK: return A_CONT;
    case OP_IN:
        if (ctl_.in_avail) {
            ctl_.in_avail = false;
            if (I.dst) set_loc(A, loc_[INL()]);
            set_loc(INL(), vdead());
            retire();
        }
        return A_CONT;
    case OP_POP: {
        const int s = I.arg;
        if (ctl_.depth[s] == 0) {
            if (!dyn(s)) return A_CONT; // empty: blocks
            const Val D = loc_[DEP(s)];
            if (D.kind == K_CONST && D.c == 0) return A_CONT;
            if (D.kind == K_REG && ctl_.lo[s] == 0) {
                if (!inline_pop_check(s)) return A_EXIT;
            }
            const Val D2 = loc_[DEP(s)]; // in its home now
            // the memory part holds at least one entry: DEP -= 1, read slot DEP
            if (D2.kind == K_CONST) {
                set_loc(DEP(s), vconst(D2.c - 1));
            } else {
                dep_add(s, -1);
                ctl_.lo[s]--;
            }
            if (I.dst) {
                const int r = fresh_reg();
                ld_entry(s, 0, r);
                Val nv;
                nv.kind = K_REG;
                nv.r = (uint16_t)r;
                set_loc(A, nv);
                r32_[r] = 1;
            }
            retire();
            return A_CONT;
        }
        const uint32_t d = ctl_.depth[s] - 1;
        Val e = stk_[s][d];
        if (I.dst) {
            if (e.kind == K_MEM) {
                const int r = fresh_reg();
                ld_entry(s, d, r);
                Val nv;
                nv.kind = K_REG;
                nv.r = (uint16_t)r;
                set_loc(A, nv);
                r32_[r] = 1;
            } else {
                set_loc(A, e);
            }
        }
        digest_entry(dig_[s], d, e, false);
        decref(e);
        stk_[s].pop_back();
        ctl_.depth[s] = d;
        retire();
        return A_CONT;
    }
    default: break;
    }
    // ops with a source operand
    const bool pn = (ctl_.pend >> n) & 1u;
    Val v;
    bool consumed = false;
    if (pn) {
        v = loc_[PENDV(n)];
    } else if (I.src == SRC_IMM) {
        v = vconst(I.imm);
    } else if (I.src == SRC_ACC) {
        v = loc_[A];
    } else if (I.src == SRC_NIL) {
        v = vconst(0);
    } else {
        const int slot = n * 4 + (I.src - SRC_R0);
        if (!((ctl_.pfull >> slot) & 1ull)) return A_CONT; // receive blocks
        v = loc_[PORT(slot)];
        ctl_.pfull &= ~(1ull << slot);
        consumed = true;
    }
    incref(v); // hold the operand for the duration of this attempt
    if (consumed) set_loc(PORT(n * 4 + (I.src - SRC_R0)), vdead());
    int rc = A_CONT;
    switch (I.op) {
    case OP_MOV:
        if (I.dst) set_loc(A, v);
        retire();
        break;
    case OP_ADD: op_addsub(A, loc_[A], v, false); retire(); break;
    case OP_SUB: op_addsub(A, loc_[A], v, true); retire(); break;
    case OP_JRO:
        if (v.kind == K_CONST) {
            int64_t t = wadd((int64_t)ip, v.c);
            t = std::min<int64_t>(std::max<int64_t>(t, 0), (int64_t)len - 1);
            jump((uint32_t)t);
        } else {
            exit_jro(n, v);
            rc = A_EXIT;
        }
        break;
    case OP_SEND: {
        const int slot = I.arg;
        if (!((ctl_.pfull >> slot) & 1ull)) {
            set_loc(PORT(slot), trunc(v));
            ctl_.pfull |= 1ull << slot;
            ctl_.pend &= ~(1u << n);
            set_loc(PENDV(n), vdead());
            retire();
        } else if (!pn) {
            ctl_.pend |= 1u << n;
            set_loc(PENDV(n), trunc(v));
            ctl_.changed = true;
        }
        break;
    }
    case OP_OUT:
        if (sess_) { // outChan <- v blocks while full (master.go:246, capacity 1 :59)
            if (!ctl_.out_cnt) {
                set_loc(OUTL(), trunc(v));
                ctl_.out_cnt = 1;
                ctl_.pend &= ~(1u << n);
                set_loc(PENDV(n), vdead());
                retire();
            } else if (!pn) {
                ctl_.pend |= 1u << n;
                set_loc(PENDV(n), trunc(v));
                ctl_.changed = true;
            }
            break;
        }
        if (ctl_.out_cnt < 2) {
            if (ctl_.out_cnt == 0) set_loc(OUTL(), trunc(v));
            ctl_.out_cnt++;
            ctl_.pend &= ~(1u << n);
            set_loc(PENDV(n), vdead());
            retire();
            if (soo_) {
                exit_end(MK_ST_OUTPUT_STOP);
                rc = A_EXIT;
            }
        } else if (!pn) {
            ctl_.pend |= 1u << n;
            set_loc(PENDV(n), trunc(v));
            ctl_.changed = true;
        }
        break;
    case OP_PUSH: {
        const int s = I.arg;
        const Val D = dyn(s) ? loc_[DEP(s)] : vconst(0);
        const int64_t known = (D.kind == K_CONST ? D.c : (int64_t)ctl_.lo[s]) + ctl_.depth[s];
        if (known >= (int64_t)cap_) {
            exit_end(MK_ST_STACK_OVERFLOW);
            rc = A_EXIT;
            break;
        }
        if (D.kind == K_REG) { // the lane overflows here iff DEP >= cap - depth
            const Val o = out_val();
            const uint8_t st = MK_ST_STACK_OVERFLOW | out_bit();
            const uint64_t lim = cap_ - ctl_.depth[s];
            if (o.kind == K_REG) emit(U_OVF, (uint8_t)(UF_OUTREG | fa(o)), st, o.r, D.r, 0);
            else emit(U_OVF, 0, st, 0, D.r, o.kind == K_CONST ? o.c : 0);
            emit_ext((int64_t)(((uint64_t)lim << 32) | steps_));
        }
        const Val e = trunc(v);
        incref(e);
        stk_[s].push_back(e);
        digest_entry(dig_[s], ctl_.depth[s], e, true);
        ctl_.depth[s]++;
        retire();
        break;
    }
    case OP_HANG:
        ctl_.hung |= 1u << n;
        ctl_.changed = true;
        break;
    case OP_RETRY:
        if (consumed) ctl_.changed = true;
        break;
    default: break;
    }
    decref(v);
    return rc;
}

void Compiler::compile_entry(uint32_t id)
{
    load_entry(id);
    std::unordered_set<std::string> seen;
    size_t last_size = 0;
    uint32_t idle = 0;
    bool done = sess_ && ctl_.pre && session_round_start(); // a call's first round start
    for (; !done;) {
        if (fail_) return;
        if (ctl_.pos == N_) {
            if (!ctl_.changed) {
                if (sess_) exit_yield(MK_ST_QUIESCENT); // the call closes; the instance lives on
                else exit_end(MK_ST_QUIESCENT);
                break;
            }
            if (sess_) { // session_step: deposit, take, then the budget check
                ctl_.pos = 0;
                ctl_.changed = false;
                if (session_round_start()) break;
                round_end_marker();
            } else {
                round_end_marker();
            }
            ctl_.pos = 0;
            ctl_.changed = false;
            if (++rounds_ > lim_.max_rounds) { failf("symbolic round budget exceeded"); return; }
            prune(ctl_, loc_);
            // prune() drops references without decref: rebuild the counts
            std::fill(refcnt_.begin(), refcnt_.end(), 0);
            for (int X = 0; X < L0_; X++) incref(loc_[X]);
            for (int s = 0; s < S_; s++)
                for (const Val &e : stk_[s]) incref(e);
            const std::string k = key_of(ctl_, loc_, dig_);
            if (memo_.count(k) || seen.count(k) || code_.size() > lim_.max_sb_uops) {
                exit_jump();
                break;
            }
            seen.insert(k);
            // a round that emitted nothing but its own ROUND_END marker (2 words) is idle
            idle = (code_.size() <= last_size + 2) ? idle + 1 : 0;
            if (idle > lim_.idle_rounds) {
                generalize();
                idle = 0;
            }
            last_size = code_.size();
            continue;
        }
        if (attempt(ctl_.pos) == A_EXIT) break;
        ctl_.pos++;
    }
    if (fail_) return;
    total_words_ += (uint32_t)code_.size() + 1;
    if (total_words_ > lim_.max_uops) { failf("micro-op budget exceeded"); return; }
    if (sb_code_.size() <= id) sb_code_.resize(id + 1);
    sb_code_[id] = std::move(code_);
    code_.clear();
}

// Slot sharing (the memory analogue of register allocation).  An ordinary
// stack's entry at depth d has one slot for the whole program (slot_of), so
// the slot count is the sum of every stack's deepest spill -- C4's eight
// stacks take 8 x 41 slots at D = 64 although node k drains its stack before
// node k + 1 pushes (stack.go:95-155 moves nothing between the stacks).
// On one lane a stack's slots hold data at most between its first and last
// slot access; two stacks may share memory when those windows never overlap
// on any lane.  A lane runs a superblock front to back (a side exit only
// skips the rest) and its superblocks one after another, so the windows of
// A and B overlap on a lane's path only if some access to B lies between two
// accesses to A (or the reverse).  So A and B interfere when an access to B
// can be reached from an access to A and can reach one (may-analyses over
// the superblock graph, loops included: accessed before / after a point on
// some path; a loop that touches A makes A live all through it).  Stacks
// that do not interfere share a slot range (greedy colouring; slot = range
// base + depth, affine in the depth, so tis_jit's loop rolling still sees
// the same runs).  Dynamic stacks keep their ranges [k*cap, (k+1)*cap).
// MK_SCHED_SHARE=0 turns the pass off (SchedLimits::share_slots).
void Compiler::share_slots()
{
    if (!lim_.share_slots || !any_slot_ || max_slot_ < 2) return;
    const size_t nsb = sb_code_.size();
    auto two_words = [](uint8_t op) {
        return op == U_BR || op == U_JRO || op == U_END || op == U_ROUND_END || op == U_OVF || op == U_BRX ||
               op == U_YIELD;
    };
    // superblock successors (exits and side exits)
    std::vector<std::vector<uint32_t>> succ(nsb);
    for (size_t id = 0; id < nsb; id++) {
        const std::vector<UOp> &sc = sb_code_[id];
        for (size_t i = 0; i < sc.size(); i++) {
            const UOp &u = sc[i];
            // a session's next call goes on with the state a yield leaves
            if (u.op == U_JUMP || u.op == U_BRX || u.op == U_YIELD) succ[id].push_back((uint32_t)(u.imm / 2));
            else if (u.op == U_BR) {
                succ[id].push_back((uint32_t)((uint64_t)u.imm & 0xFFFFFFFFu) / 2);
                succ[id].push_back((uint32_t)((uint64_t)u.imm >> 32) / 2);
            } else if (u.op == U_JRO) {
                for (uint32_t t = 0; t <= u.b; t++) succ[id].push_back(jtab_[(size_t)u.imm + t] / 2);
            }
            if (two_words(u.op)) i++;
        }
    }
    for (auto &v : succ)
        for (uint32_t t : v)
            if (t >= nsb) return;
    // static slot -> (stack, depth)
    std::vector<int> st_of(max_slot_, -1);
    std::vector<uint32_t> d_of(max_slot_, 0);
    for (int s = 0; s < (int)slot_id_.size(); s++)
        for (uint32_t d = 0; d < slot_id_[s].size(); d++)
            if (slot_id_[s][d] >= 0) st_of[slot_id_[s][d]] = s, d_of[slot_id_[s][d]] = d;
    const uint32_t base0 = ndyn_ * cap_;
    auto stack_of = [&](const UOp &u) {
        uint32_t slot;
        if (u.op == U_ST || u.op == U_LD) slot = (uint32_t)u.imm;
        else if (u.op == U_STI) slot = (uint32_t)u.a | ((uint32_t)u.b << 16);
        else return -1;
        return slot >= base0 && slot - base0 < max_slot_ ? st_of[slot - base0] : -2;
    };
    // per superblock: first / last access position of each stack; the size of each stack's range
    const size_t S = (size_t)S_;
    std::vector<int64_t> first(nsb * S, -1), last(nsb * S, -1);
    std::vector<uint32_t> size(S, 0);
    for (size_t id = 0; id < nsb; id++)
        for (size_t i = 0; i < sb_code_[id].size(); i++) {
            const UOp &u = sb_code_[id][i];
            const int s = stack_of(u);
            if (s == -2) return; // a slot no stack owns: leave everything alone
            if (s >= 0) {
                if (first[id * S + s] < 0) first[id * S + s] = (int64_t)i;
                last[id * S + s] = (int64_t)i;
                const uint32_t slot = u.op == U_STI ? ((uint32_t)u.a | ((uint32_t)u.b << 16)) : (uint32_t)u.imm;
                size[s] = std::max(size[s], d_of[slot - base0] + 1);
            }
            if (two_words(u.op)) i++;
        }
    // may-analyses to a fixpoint (loops included): stacks accessed on some
    // path before a superblock's entry / after its exits, as 64-bit sets,
    // propagated by worklists (a set only grows, so each superblock is
    // revisited at most S times)
    if (S > 64) return;
    std::vector<uint64_t> acc(nsb, 0), bef(nsb, 0), aft(nsb, 0);
    for (size_t id = 0; id < nsb; id++)
        for (size_t s = 0; s < S; s++)
            if (first[id * S + s] >= 0) acc[id] |= 1ull << s;
    std::vector<std::vector<uint32_t>> pred(nsb);
    for (uint32_t id = 0; id < nsb; id++)
        for (uint32_t t : succ[id]) pred[t].push_back(id);
    std::vector<uint32_t> work;
    std::vector<uint8_t> queued(nsb, 1);
    for (uint32_t id = 0; id < nsb; id++) work.push_back(id);
    while (!work.empty()) { // forward: bef[t] |= bef[id] | acc[id]
        const uint32_t id = work.back();
        work.pop_back();
        queued[id] = 0;
        for (uint32_t t : succ[id]) {
            const uint64_t n = bef[t] | bef[id] | acc[id];
            if (n != bef[t]) {
                bef[t] = n;
                if (!queued[t]) queued[t] = 1, work.push_back(t);
            }
        }
    }
    std::fill(queued.begin(), queued.end(), 1);
    for (uint32_t id = 0; id < nsb; id++) work.push_back(id);
    while (!work.empty()) { // backward: aft[p] |= aft[id] | acc[id]
        const uint32_t id = work.back();
        work.pop_back();
        queued[id] = 0;
        for (uint32_t q : pred[id]) {
            const uint64_t n = aft[q] | aft[id] | acc[id];
            if (n != aft[q]) {
                aft[q] = n;
                if (!queued[q]) queued[q] = 1, work.push_back(q);
            }
        }
    }
    // A and B interfere when an access to B has A accessed before it and after it
    std::vector<uint8_t> clash(S * S, 0);
    for (size_t id = 0; id < nsb; id++)
        for (size_t i = 0; i < sb_code_[id].size(); i++) {
            const UOp &u = sb_code_[id][i];
            const int b = stack_of(u);
            if (b >= 0)
                for (size_t a = 0; a < S; a++) {
                    if ((int)a == b || clash[a * S + b]) continue;
                    const bool pre = ((bef[id] >> a) & 1u) || (first[id * S + a] >= 0 && first[id * S + a] < (int64_t)i);
                    const bool post = ((aft[id] >> a) & 1u) || last[id * S + a] > (int64_t)i;
                    if (pre && post) clash[a * S + b] = clash[b * S + a] = 1;
                }
            if (two_words(u.op)) i++;
        }
    // greedy colouring, largest ranges first: a stack joins the first range
    // none of whose stacks it interferes with
    std::vector<int> by_size;
    for (size_t s = 0; s < S; s++)
        if (size[s]) by_size.push_back((int)s);
    std::stable_sort(by_size.begin(), by_size.end(), [&](int a, int b) { return size[a] > size[b]; });
    std::vector<std::vector<int>> ranges;
    std::vector<uint32_t> range_size, range_of(S, 0);
    for (int s : by_size) {
        size_t r = 0;
        for (; r < ranges.size(); r++) {
            bool ok = true;
            for (int o : ranges[r]) ok = ok && !clash[(size_t)o * S + s];
            if (ok) break;
        }
        if (r == ranges.size()) ranges.emplace_back(), range_size.push_back(0);
        ranges[r].push_back(s);
        range_size[r] = std::max(range_size[r], size[s]);
        range_of[s] = (uint32_t)r;
    }
    std::vector<uint32_t> range_base(range_size.size(), 0);
    uint32_t total = 0;
    for (size_t r = 0; r < range_size.size(); r++) range_base[r] = total, total += range_size[r];
    if (total >= max_slot_) return; // nothing shared
    for (auto &sc : sb_code_)
        for (size_t i = 0; i < sc.size(); i++) {
            UOp &u = sc[i];
            if (stack_of(u) >= 0) {
                const uint32_t slot = u.op == U_STI ? ((uint32_t)u.a | ((uint32_t)u.b << 16)) : (uint32_t)u.imm;
                const uint32_t k = slot - base0, ns = base0 + range_base[range_of[st_of[k]]] + d_of[k];
                if (u.op == U_STI) u.a = (uint16_t)(ns & 0xFFFF), u.b = (uint16_t)(ns >> 16);
                else u.imm = ns;
            }
            if (two_words(u.op)) i++;
        }
    for (int s = 0; s < (int)slot_id_.size(); s++)
        for (uint32_t d = 0; d < slot_id_[s].size(); d++)
            if (slot_id_[s][d] >= 0) slot_id_[s][d] = (int32_t)(range_base[range_of[s]] + d);
    max_slot_ = total;
}

bool Compiler::run(SchedProgram &out, std::string &why)
{
    if (N_ > 32) { why = "too many program nodes for the compiler"; return false; }
    liveness();
    // entry state: post-/reset, post-/run, input deposited (in register 0)
    Ctl c;
    c.ip.assign(N_, 0);
    c.depth.assign(S_, 0);
    c.lo.assign(S_, 0);
    if (sess_) { // a session at the start of its first call: inChan and outChan empty
        c.in_avail = false;
        c.pre = true;
    }
    ctl_ = c;
    loc_.assign(L0_, vdead());
    for (int s = 0; s < S_; s++) loc_[DEP(s)] = vconst(0);
    for (int n = 0; n < N_; n++) {
        loc_[ACC(n)] = vconst(0);
        loc_[BAK(n)] = vconst(0);
    }
    if (!sess_) loc_[OUTL()] = vconst(0);
    stk_.assign(S_, {});
    dig_.assign(S_, StackDigest());
    ensure_reg(0);
    const int inloc = sess_ ? CIN() : INL(); // the input's location: a call's input / inChan
    home_[inloc] = 0;
    claimed_[0] = 1;
    Val in;
    in.kind = K_REG;
    in.r = 0;
    loc_[inloc] = in;
    prune(ctl_, loc_);
    get_or_create(ctl_, loc_);
    while (!work_.empty() && !fail_) {
        const uint32_t id = work_.front();
        work_.pop_front();
        compile_entry(id);
    }
    if (fail_) {
        why = why_;
        return false;
    }
    share_slots();
    // assemble: per superblock a fast variant (GUARD + code without budget
    // markers) and a checked variant (with markers)
    out = SchedProgram();
    out.entry.assign(2 * entries_.size(), 0);
    for (size_t id = 0; id < entries_.size(); id++) {
        const std::vector<UOp> &sc = sb_code_[id];
        int64_t maxinc = -1;
        for (size_t i = 0; i < sc.size(); i++) {
            if (sc[i].op == U_ROUND_END) {
                maxinc = std::max<int64_t>(maxinc, sc[i + 1].imm);
                i++;
            } else if (sc[i].op == U_BR || sc[i].op == U_JRO || sc[i].op == U_END || sc[i].op == U_OVF ||
                       sc[i].op == U_BRX || sc[i].op == U_YIELD) {
                i++;
            }
        }
        out.entry[2 * id] = (uint32_t)out.code.size();
        if (maxinc >= 0) {
            UOp g{};
            g.op = U_GUARD;
            g.d = (uint16_t)(maxinc & 0xFFFF);
            g.a = (uint16_t)(maxinc >> 16);
            g.imm = 2 * (int64_t)id + 1;
            out.code.push_back(g);
        }
        for (size_t i = 0; i < sc.size(); i++) {
            if (sc[i].op == U_ROUND_END) { i++; continue; }
            out.code.push_back(sc[i]);
        }
        if (maxinc >= 0 && sess_) { // sessions: the interpreter runs the rest of the call
            out.entry[2 * id + 1] = (uint32_t)out.code.size();
            UOp h{};
            h.op = U_HANDOFF;
            h.imm = 2 * (int64_t)id;
            out.code.push_back(h);
        } else if (maxinc >= 0) {
            out.entry[2 * id + 1] = (uint32_t)out.code.size();
            out.code.insert(out.code.end(), sc.begin(), sc.end());
        } else {
            out.entry[2 * id + 1] = out.entry[2 * id];
        }
    }
    out.jtab = jtab_;
    out.nregs = std::max<uint32_t>(max_reg_, 1);
    out.nslots = any_slot_ ? ndyn_ * cap_ + max_slot_ : 0;
    out.ndyn = ndyn_;
    out.in_reg = 0;
    out.nsb = (uint32_t)entries_.size();
    out.sym_rounds = rounds_;
    if (sess_) {
        out.session = true;
        out.nloc = (uint32_t)L0_;
        out.dyn_base = dyn_base_;
        out.smap.resize(entries_.size());
        for (size_t id = 0; id < entries_.size(); id++) {
            const EntryState &e = entries_[id];
            SessEntry &m = out.smap[id];
            m.ip = e.ctl.ip;
            m.pend = e.ctl.pend;
            m.hung = e.ctl.hung;
            m.pfull = e.ctl.pfull;
            m.in_avail = e.ctl.in_avail;
            m.out_full = e.ctl.out_cnt != 0;
            m.deposited = e.ctl.cdep;
            m.pos = e.ctl.pos;
            m.changed = e.ctl.changed;
            m.pre = e.ctl.pre;
            m.loc.resize(L0_);
            for (int X = 0; X < L0_; X++) {
                const Val &v = e.loc[X];
                if (v.kind == K_CONST) m.loc[X].kind = 1, m.loc[X].c = v.c;
                else if (v.kind == K_REG) m.loc[X].kind = 2, m.loc[X].r = v.r;
            }
            m.stk.resize(S_);
            for (int s = 0; s < S_; s++) {
                if (dyn(s)) continue;
                for (uint32_t d = 0; d < (uint32_t)e.stk[s].size(); d++) {
                    const Val &v = e.stk[s][d];
                    SessSrc x;
                    if (v.kind == K_CONST) x.kind = 1, x.c = v.c;
                    else x.kind = 3, x.r = ndyn_ * cap_ + (uint32_t)slot_id_[s][d];
                    m.stk[s].push_back(x);
                }
            }
        }
    }
    return true;
}

} // namespace

// MK_SCHED_WIDEN / MK_SCHED_DYN / MK_SCHED_MAX_SB / MK_SCHED_SOFT_REGS
// override the widening threshold, the dynamic-stack trigger, the superblock
// limit and the registers kept before stack entries spill (experiments and
// tests; unset = the caller's limits).
SchedLimits lim_env(SchedLimits lim)
{
    if (const char *e = getenv("MK_SCHED_WIDEN")) lim.widen_after = (uint32_t)atoi(e);
    if (const char *e = getenv("MK_SCHED_DYN")) lim.dyn_depths = (uint32_t)atoi(e);
    if (const char *e = getenv("MK_SCHED_MAX_SB")) lim.max_superblocks = (uint32_t)atoi(e);
    if (const char *e = getenv("MK_SCHED_SHARE")) lim.share_slots = atoi(e) != 0;
    if (const char *e = getenv("MK_SCHED_MAX_REGS")) {
        const int v = atoi(e);
        if (v >= 8 && v <= 1024) lim.max_regs = (uint32_t)v;
    }
    if (const char *e = getenv("MK_SCHED_SOFT_REGS")) {
        const int v = atoi(e);
        if (v >= 4 && (uint32_t)v < lim.max_regs) lim.soft_regs = (uint32_t)v;
    }
    return lim;
}

namespace {
bool compile_any(const Network &net, uint32_t stack_cap, bool stop_on_output, bool sess, const SchedLimits &lim,
                 SchedProgram &out, std::string &why)
{
    if (net.uses_remote) { // X-ops wait on the host: only the interpreters run them
        why = "network addresses remote peers (MK_NODE_REMOTE_*)";
        return false;
    }
    // A stack whose depth follows the data is found by compiling: the
    // compile stops at the first such stack and is repeated with it dynamic.
    const int S = net.uses_stacks ? net.nstack : 0;
    std::vector<uint8_t> dyn(S, 0);
    const SchedLimits L = lim_env(lim);
    for (;;) {
        Compiler c(net, stack_cap, stop_on_output, L, dyn, sess);
        if (c.run(out, why)) return true;
        bool more = false;
        for (int s = 0; s < S; s++)
            if (c.want_dyn()[s] && !dyn[s]) dyn[s] = 1, more = true;
        if (!more) return false;
    }
}
} // namespace

bool compile_schedule(const Network &net, uint32_t stack_cap, bool stop_on_output, const SchedLimits &lim,
                      SchedProgram &out, std::string &why)
{
    return compile_any(net, stack_cap, stop_on_output, false, lim, out, why);
}

bool compile_session_schedule(const Network &net, uint32_t stack_cap, const SchedLimits &lim, SchedProgram &out,
                              std::string &why)
{
    return compile_any(net, stack_cap, false, true, lim, out, why);
}

std::vector<DOp> assemble_device(const SchedProgram &p, uint32_t reg_bytes, std::vector<uint32_t> &entry_out)
{
    std::vector<DOp> out;
    std::vector<uint32_t> map(p.code.size() + 1, 0);
    const uint32_t scale = reg_bytes;
    for (size_t i = 0; i < p.code.size(); i++) {
        map[i] = (uint32_t)out.size();
        const UOp &u = p.code[i];
        DOp o{};
        o.op = u.op;
        o.fl = u.fl;
        o.imm = u.imm;
        const bool two = u.op == U_BR || u.op == U_JRO || u.op == U_END || u.op == U_ROUND_END || u.op == U_OVF ||
                         u.op == U_BRX || u.op == U_YIELD;
        const uint32_t ext = two ? (uint32_t)p.code[i + 1].imm : 0;
        switch (u.op) {
        case U_MOV: case U_ADDI: case U_RSUBI:
            o.d = u.d * scale; o.a = u.a * scale; break;
        case U_ADD: case U_SUB:
            o.d = u.d * scale; o.a = u.a * scale; o.b = u.b * scale; break;
        case U_LI: case U_LD:
            o.d = u.d * scale; break;
        case U_ST:
            o.a = u.a * scale; break;
        case U_STI:
            o.d = (uint32_t)u.a | ((uint32_t)u.b << 16); break;
        case U_JUMP: case U_GUARD:
            o.inc = (uint32_t)u.d | ((uint32_t)u.a << 16); break;
        case U_BR: case U_BRX:
            o.a = u.a * scale; o.inc = ext; break;
        case U_JRO:
            o.d = u.d; o.a = u.a * scale; o.b = u.b; o.inc = ext; break;
        case U_END: case U_ROUND_END:
            o.d = u.d; o.a = (u.fl & UF_OUTREG) ? u.a * scale : 0; o.inc = ext; break;
        case U_STX:
            o.a = u.a * scale; o.b = u.b * scale; break;
        case U_LDX:
            o.d = u.d * scale; o.b = u.b * scale; break;
        case U_YIELD: { // imm = next variant | out constant << 32, inc = steps
            const uint64_t x = (uint64_t)p.code[i + 1].imm;
            o.d = u.d;
            o.a = (u.fl & UF_OUTREG) ? u.a * scale : 0;
            o.inc = (uint32_t)x;
            o.imm = (int64_t)(((x >> 32) << 32) | (uint32_t)u.imm);
            break;
        }
        case U_OVF: {
            const uint64_t x = (uint64_t)p.code[i + 1].imm;
            o.d = u.d;
            o.a = (u.fl & UF_OUTREG) ? u.a * scale : 0;
            o.b = u.b * scale;
            o.inc = (uint32_t)x;
            o.imm = (int64_t)(((x >> 32) << 32) | (uint32_t)(int32_t)u.imm);
            break;
        }
        default: break;
        }
        out.push_back(o);
        if (two) i++;
    }
    map[p.code.size()] = (uint32_t)out.size();
    entry_out.resize(p.entry.size());
    for (size_t v = 0; v < p.entry.size(); v++) entry_out[v] = map[p.entry[v]];
    return out;
}

void build_sess_map(const SchedProgram &p, int nprog, int nstack, std::vector<SessMapHdr> &hdr,
                    std::vector<SessSrcDev> &rec)
{
    hdr.clear();
    rec.clear();
    auto put = [&](const SessSrc &x) { rec.push_back(SessSrcDev{x.c, x.r, x.kind}); };
    for (const SessEntry &m : p.smap) {
        SessMapHdr h{};
        h.off = (uint32_t)rec.size();
        h.pend = m.pend;
        h.hung = m.hung;
        h.pfull = m.pfull;
        h.flags = (m.in_avail ? 1u : 0u) | (m.out_full ? 2u : 0u) | (m.deposited ? 4u : 0u) | (m.changed ? 8u : 0u) |
                  (m.pre ? 16u : 0u) | (uint32_t)m.pos << 8;
        hdr.push_back(h);
        for (int n = 0; n < nprog; n++) rec.push_back(SessSrcDev{(int64_t)m.ip[n], 0u, 1u});
        for (const SessSrc &x : m.loc) put(x);
        for (int s = 0; s < nstack; s++) {
            const size_t k = (size_t)s < m.stk.size() ? m.stk[s].size() : 0;
            rec.push_back(SessSrcDev{(int64_t)k, 0u, 1u});
            for (size_t d = 0; d < k; d++) put(m.stk[s][d]);
        }
    }
}

std::string sched_disasm(const SchedProgram &p)
{
    static const char *names[U_COUNT] = {"MOV", "LI",  "ADD", "SUB", "ADDI",  "RSUBI",     "ST",  "STI", "LD",
                                         "STX", "LDX", "JUMP", "BR", "JRO", "END", "GUARD", "ROUND_END", "OVF",
                                         "BRX", "YIELD", "HANDOFF"};
    std::string s;
    char buf[200];
    snprintf(buf, sizeof buf, "superblocks=%u regs=%u slots=%u words=%zu jtab=%zu\n", p.nsb, p.nregs, p.nslots,
             p.code.size(), p.jtab.size());
    s += buf;
    std::vector<int> starts(p.code.size() + 1, -1);
    for (size_t v = 0; v < p.entry.size(); v++)
        if (starts[p.entry[v]] < 0) starts[p.entry[v]] = (int)v;
    for (size_t i = 0; i < p.code.size(); i++) {
        if (starts[i] >= 0) {
            snprintf(buf, sizeof buf, "sb%d%s:\n", starts[i] / 2, (starts[i] & 1) ? " (checked)" : "");
            s += buf;
        }
        const UOp &u = p.code[i];
        const char *nm = u.op < U_COUNT ? names[u.op] : "?";
        snprintf(buf, sizeof buf, "  %5zu %-9s fl=%02x d=%u a=%u b=%u imm=%lld\n", i, nm, u.fl, u.d, u.a, u.b,
                 (long long)u.imm);
        s += buf;
        if (u.op == U_BR || u.op == U_JRO || u.op == U_END || u.op == U_ROUND_END || u.op == U_OVF || u.op == U_BRX ||
            u.op == U_YIELD) {
            i++;
            snprintf(buf, sizeof buf, "        ext       steps+=%lld\n", (long long)p.code[i].imm);
            s += buf;
        }
    }
    return s;
}

} // namespace mk
