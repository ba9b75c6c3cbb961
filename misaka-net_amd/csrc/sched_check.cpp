// sched_check.cpp -- host model of the tier-2 superblock executor
// (tis_sched_exec in mk_exec.hip), built into a separate CHECK library
// (lib/libmisaka_amd_check.so) so the schedule compiler can be fuzzed against
// the CPU oracle without a GPU.  It is not part of the product library and
// no product entry point can reach it.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mk.h"
#include "../../oracle/orc_flat.h"
#include "tis_front.h"
#include "tis_jit.h"
#include "tis_sched.h"
#include "sess_convert.h"

namespace {

struct CheckNet {
    mk::Network net;
};

inline int64_t sx(int64_t v, bool t) { return t ? (int64_t)(int32_t)(uint32_t)(uint64_t)v : v; }

} // namespace

extern "C" {

void *mkc_load(const mk_node_desc *nodes, int n, char *err, size_t err_len)
{
    std::vector<mk::NodeSpec> specs;
    for (int i = 0; i < n; i++) specs.push_back({nodes[i].name, nodes[i].kind, nodes[i].program ? nodes[i].program : ""});
    auto *h = new CheckNet();
    std::string e;
    if (mk::lower_network(specs, h->net, e)) {
        snprintf(err, err_len, "%s", e.c_str());
        delete h;
        return nullptr;
    }
    return h;
}

void mkc_free(void *h) { delete (CheckNet *)h; }

// Returns 0 when compiled and emulated, 1 when the compiler declined (why),
// negative on error.  plan (nullable) receives the disassembly.
int mkc_emulate(void *hv, uint32_t budget, uint32_t cap, int soo, const int64_t *in, size_t n, int32_t *out,
                uint8_t *status, uint32_t *steps_out, char *why, size_t why_len, char *plan, size_t plan_len)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w;
    mk::SchedLimits lim;
    if (!mk::compile_schedule(h->net, cap, soo != 0, lim, P, w)) {
        snprintf(why, why_len, "%s", w.c_str());
        return 1;
    }
    if (plan && plan_len) snprintf(plan, plan_len, "%s", mk::sched_disasm(P).c_str());
    // execute the device form (one lane, one slot: register byte offsets are r * 8)
    std::vector<uint32_t> entry;
    const std::vector<mk::DOp> D = mk::assemble_device(P, 8, entry);
    std::vector<int64_t> R(P.nregs);
    std::unordered_map<uint32_t, int32_t> slots;
    auto reg = [&](uint32_t off) -> int64_t & { return R.at(off / 8); };
    for (size_t i = 0; i < n; i++) {
        std::fill(R.begin(), R.end(), (int64_t)0x5A5A5A5A5A5A5A5All); // stale register contents
        slots.clear();
        R[P.in_reg] = (int32_t)in[i];
        uint32_t sb = 0, steps = 0, st = 0;
        int32_t outv = 0;
        bool done = false;
        uint64_t guard_words = 0;
        const char *tr = getenv("MKC_TRACE"); // debugging: trace lane i's superblocks
        const bool trace = tr && (size_t)atoll(tr) == i;
        while (!done) {
            uint32_t pc = entry[sb];
            if (trace) {
                fprintf(stderr, "sb%u%s steps=%u R:", sb / 2, (sb & 1) ? "c" : "", steps);
                for (size_t r = 0; r < R.size(); r++) fprintf(stderr, " %lld", (long long)R[r]);
                fprintf(stderr, "\n");
            }
            for (;;) {
                if (++guard_words > (1ull << 34)) return -2; // runaway
                const mk::DOp &I = D.at(pc);
                bool leave = false;
                const bool ta = I.fl & mk::UF_TA, tb = I.fl & mk::UF_TB;
                switch (I.op) {
                case mk::U_MOV: reg(I.d) = sx(reg(I.a), ta); pc++; break;
                case mk::U_LI: reg(I.d) = I.imm; pc++; break;
                case mk::U_ADD: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) + (uint64_t)sx(reg(I.b), tb)); pc++; break;
                case mk::U_SUB: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) - (uint64_t)sx(reg(I.b), tb)); pc++; break;
                case mk::U_ADDI: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) + (uint64_t)I.imm); pc++; break;
                case mk::U_RSUBI: reg(I.d) = (int64_t)((uint64_t)I.imm - (uint64_t)sx(reg(I.a), ta)); pc++; break;
                case mk::U_ST: slots[(uint32_t)I.imm] = (int32_t)sx(reg(I.a), ta); pc++; break;
                case mk::U_STI: slots[I.d] = (int32_t)I.imm; pc++; break;
                case mk::U_LD: {
                    auto it = slots.find((uint32_t)I.imm);
                    if (it == slots.end()) return -3; // load of a slot never stored
                    reg(I.d) = it->second;
                    pc++;
                    break;
                }
                case mk::U_STX: {
                    const int64_t x = reg(I.b);
                    if (x < 0 || (uint64_t)I.imm + (uint64_t)x >= P.nslots) return -5; // index out of range
                    slots[(uint32_t)(I.imm + x)] = (int32_t)sx(reg(I.a), ta);
                    pc++;
                    break;
                }
                case mk::U_LDX: {
                    const int64_t x = reg(I.b);
                    if (x < 0 || (uint64_t)I.imm + (uint64_t)x >= P.nslots) return -5;
                    auto it = slots.find((uint32_t)(I.imm + x));
                    if (it == slots.end()) return -3;
                    reg(I.d) = it->second;
                    pc++;
                    break;
                }
                case mk::U_BRX: {
                    const int64_t v = sx(reg(I.a), ta);
                    const uint32_t c = (I.fl >> mk::UF_COND_SHIFT) & 3u;
                    const bool take = c == 0 ? v == 0 : c == 1 ? v != 0 : c == 2 ? v > 0 : v < 0;
                    if (take) {
                        steps += I.inc;
                        sb = (uint32_t)I.imm;
                        leave = true;
                    }
                    pc++;
                    break;
                }
                case mk::U_OVF:
                    if ((uint64_t)reg(I.b) >= ((uint64_t)I.imm >> 32)) {
                        steps += I.inc;
                        outv = (I.fl & mk::UF_OUTREG) ? (int32_t)sx(reg(I.a), ta) : (int32_t)(uint32_t)(uint64_t)I.imm;
                        st = I.d;
                        done = leave = true;
                    }
                    pc++;
                    break;
                case mk::U_JUMP: steps += I.inc; sb = (uint32_t)I.imm; leave = true; break;
                case mk::U_BR: {
                    const int64_t v = sx(reg(I.a), ta);
                    const uint32_t c = (I.fl >> mk::UF_COND_SHIFT) & 3u;
                    const bool take = c == 0 ? v == 0 : c == 1 ? v != 0 : c == 2 ? v > 0 : v < 0;
                    steps += I.inc;
                    sb = take ? (uint32_t)(uint64_t)I.imm : (uint32_t)((uint64_t)I.imm >> 32);
                    leave = true;
                    break;
                }
                case mk::U_JRO: {
                    int64_t t = (int64_t)((uint64_t)I.d + (uint64_t)sx(reg(I.a), ta));
                    t = t > (int64_t)I.b ? (int64_t)I.b : t;
                    t = t < 0 ? 0 : t;
                    steps += I.inc;
                    sb = P.jtab.at((size_t)I.imm + (size_t)t);
                    leave = true;
                    break;
                }
                case mk::U_END:
                    steps += I.inc;
                    outv = (I.fl & mk::UF_OUTREG) ? (int32_t)sx(reg(I.a), ta) : (int32_t)I.imm;
                    st = I.d;
                    done = leave = true;
                    break;
                case mk::U_GUARD:
                    if ((uint64_t)steps + I.inc >= budget) {
                        sb = (uint32_t)I.imm;
                        leave = true;
                    }
                    pc++;
                    break;
                case mk::U_ROUND_END:
                    if ((uint64_t)steps + I.inc >= budget) {
                        steps += I.inc;
                        outv = (I.fl & mk::UF_OUTREG) ? (int32_t)sx(reg(I.a), ta) : (int32_t)I.imm;
                        st = I.d;
                        done = leave = true;
                    }
                    pc++;
                    break;
                default: return -4;
                }
                if (leave) break;
            }
        }
        out[i] = (st & MK_ST_HAS_OUTPUT) ? outv : 0;
        status[i] = (uint8_t)st;
        if (steps_out) steps_out[i] = steps;
    }
    return 0;
}

// ---- stateful sessions (tis_sched.h compile_session_schedule) ----------------
// n persistent instances, one /compute call on all of them per
// mkc_sess_call, executing the session schedule's device form exactly as the
// native tier's session kernel does.  A call that hands off (U_HANDOFF: the
// budget slice ends inside a superblock) reports status 0xFE; its state, in
// the interpreter's terms (sess_convert.h), is what mkc_sess_export gives
// the oracle to finish the call (orc_session_import).
struct SessEmu {
    mk::SchedProgram P;
    std::vector<mk::DOp> D;
    std::vector<uint32_t> entry;
    std::vector<mk::SessMapHdr> hdr;
    std::vector<mk::SessSrcDev> rec;
    int N = 0, S = 0;
    uint32_t cap = 0;
    std::vector<std::vector<int64_t>> R;
    std::vector<std::unordered_map<uint32_t, int32_t>> slots;
    std::vector<uint32_t> sb;       // variant the next call starts at
    std::vector<uint8_t> state;     // 0 live, 1 ended (stack overflow), 2 handed off
    std::vector<uint32_t> hand_sb;  // superblock of the hand-off
    std::vector<uint32_t> hand_steps;
};

void *mkc_sess_new(void *hv, uint32_t cap, uint32_t n, char *why, size_t why_len)
{
    auto *h = (CheckNet *)hv;
    auto *e = new SessEmu();
    std::string w;
    mk::SchedLimits lim;
    if (!mk::compile_session_schedule(h->net, cap, lim, e->P, w)) {
        snprintf(why, why_len, "%s", w.c_str());
        delete e;
        return nullptr;
    }
    e->D = mk::assemble_device(e->P, 8, e->entry);
    e->N = h->net.nprog;
    e->S = h->net.uses_stacks ? h->net.nstack : 0;
    e->cap = cap;
    mk::build_sess_map(e->P, e->N, e->S, e->hdr, e->rec);
    e->R.assign(n, std::vector<int64_t>(e->P.nregs, (int64_t)0x5A5A5A5A5A5A5A5All));
    e->slots.assign(n, {});
    e->sb.assign(n, 0);
    e->state.assign(n, 0);
    e->hand_sb.assign(n, 0);
    e->hand_steps.assign(n, 0);
    snprintf(why, why_len, "%s", mk::sched_disasm(e->P).substr(0, why_len ? why_len - 1 : 0).c_str());
    return e;
}

void mkc_sess_free(void *ev) { delete (SessEmu *)ev; }

int mkc_sess_call(void *ev, const int64_t *in, uint32_t budget, int32_t *out, uint8_t *status, uint32_t *steps_out)
{
    auto *e = (SessEmu *)ev;
    const mk::SchedProgram &P = e->P;
    for (size_t i = 0; i < e->sb.size(); i++) {
        out[i] = 0;
        steps_out[i] = 0;
        if (e->state[i] == 1) { status[i] = MK_ST_STACK_OVERFLOW; continue; }
        if (e->state[i] == 2) { status[i] = 0xFE; continue; }
        std::vector<int64_t> &R = e->R[i];
        auto &slots = e->slots[i];
        auto reg = [&](uint32_t off) -> int64_t & { return R.at(off / 8); };
        R[P.in_reg] = (int32_t)in[i];
        uint32_t sb = e->sb[i], steps = 0;
        uint64_t words = 0;
        bool done = false;
        while (!done) {
            uint32_t pc = e->entry.at(sb);
            for (bool leave = false; !leave;) {
                if (++words > (1ull << 34)) return -2;
                const mk::DOp &I = e->D.at(pc);
                const bool ta = I.fl & mk::UF_TA, tb = I.fl & mk::UF_TB;
                switch (I.op) {
                case mk::U_MOV: reg(I.d) = sx(reg(I.a), ta); pc++; break;
                case mk::U_LI: reg(I.d) = I.imm; pc++; break;
                case mk::U_ADD: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) + (uint64_t)sx(reg(I.b), tb)); pc++; break;
                case mk::U_SUB: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) - (uint64_t)sx(reg(I.b), tb)); pc++; break;
                case mk::U_ADDI: reg(I.d) = (int64_t)((uint64_t)sx(reg(I.a), ta) + (uint64_t)I.imm); pc++; break;
                case mk::U_RSUBI: reg(I.d) = (int64_t)((uint64_t)I.imm - (uint64_t)sx(reg(I.a), ta)); pc++; break;
                case mk::U_ST: slots[(uint32_t)I.imm] = (int32_t)sx(reg(I.a), ta); pc++; break;
                case mk::U_STI: slots[I.d] = (int32_t)I.imm; pc++; break;
                case mk::U_LD: {
                    auto it = slots.find((uint32_t)I.imm);
                    if (it == slots.end()) return -3;
                    reg(I.d) = it->second;
                    pc++;
                    break;
                }
                case mk::U_STX: {
                    const int64_t x = reg(I.b);
                    if (x < 0 || (uint64_t)I.imm + (uint64_t)x >= P.nslots) return -5;
                    slots[(uint32_t)(I.imm + x)] = (int32_t)sx(reg(I.a), ta);
                    pc++;
                    break;
                }
                case mk::U_LDX: {
                    const int64_t x = reg(I.b);
                    if (x < 0 || (uint64_t)I.imm + (uint64_t)x >= P.nslots) return -5;
                    auto it = slots.find((uint32_t)(I.imm + x));
                    if (it == slots.end()) return -3;
                    reg(I.d) = it->second;
                    pc++;
                    break;
                }
                case mk::U_BRX: {
                    const int64_t v = sx(reg(I.a), ta);
                    const uint32_t c = (I.fl >> mk::UF_COND_SHIFT) & 3u;
                    const bool take = c == 0 ? v == 0 : c == 1 ? v != 0 : c == 2 ? v > 0 : v < 0;
                    if (take) {
                        steps += I.inc;
                        sb = (uint32_t)I.imm;
                        leave = true;
                    }
                    pc++;
                    break;
                }
                case mk::U_OVF:
                    if ((uint64_t)reg(I.b) >= ((uint64_t)I.imm >> 32)) {
                        steps += I.inc;
                        status[i] = (uint8_t)I.d;
                        e->state[i] = 1;
                        done = leave = true;
                    }
                    pc++;
                    break;
                case mk::U_JUMP: steps += I.inc; sb = (uint32_t)I.imm; leave = true; break;
                case mk::U_BR: {
                    const int64_t v = sx(reg(I.a), ta);
                    const uint32_t c = (I.fl >> mk::UF_COND_SHIFT) & 3u;
                    const bool take = c == 0 ? v == 0 : c == 1 ? v != 0 : c == 2 ? v > 0 : v < 0;
                    steps += I.inc;
                    sb = take ? (uint32_t)(uint64_t)I.imm : (uint32_t)((uint64_t)I.imm >> 32);
                    leave = true;
                    break;
                }
                case mk::U_JRO: {
                    int64_t t = (int64_t)((uint64_t)I.d + (uint64_t)sx(reg(I.a), ta));
                    t = t > (int64_t)I.b ? (int64_t)I.b : t;
                    t = t < 0 ? 0 : t;
                    steps += I.inc;
                    sb = P.jtab.at((size_t)I.imm + (size_t)t);
                    leave = true;
                    break;
                }
                case mk::U_END: // a stack overflow ends the session
                    steps += I.inc;
                    status[i] = (uint8_t)I.d;
                    e->state[i] = 1;
                    done = leave = true;
                    break;
                case mk::U_YIELD:
                    steps += I.inc;
                    out[i] = (I.d & MK_ST_HAS_OUTPUT)
                                 ? ((I.fl & mk::UF_OUTREG) ? (int32_t)sx(reg(I.a), ta) : (int32_t)((uint64_t)I.imm >> 32))
                                 : 0;
                    status[i] = (uint8_t)I.d;
                    e->sb[i] = (uint32_t)(uint64_t)I.imm;
                    done = leave = true;
                    break;
                case mk::U_HANDOFF:
                    status[i] = 0xFE;
                    e->state[i] = 2;
                    e->hand_sb[i] = (uint32_t)I.imm / 2;
                    e->hand_steps[i] = steps;
                    done = leave = true;
                    break;
                case mk::U_GUARD:
                    if ((uint64_t)steps + I.inc >= budget) {
                        sb = (uint32_t)I.imm;
                        leave = true;
                    }
                    pc++;
                    break;
                default: return -4;
                }
            }
        }
        steps_out[i] = steps;
    }
    return 0;
}

namespace {
struct FlatOut {
    orc_flat &f;
    int32_t *entries;
    uint32_t cap;
    void acc(int n, int64_t v) { f.acc[n] = v; }
    void bak(int n, int64_t v) { f.bak[n] = v; }
    void ip(int n, int32_t v) { f.ip[n] = v; }
    void pendv(int n, int32_t v) { f.pendv[n] = v; }
    void port(int q, int32_t v) { f.port[q] = v; }
    void pfull(uint64_t x) { f.pfull = x; }
    void bits(uint32_t pend, uint32_t hung) { f.pend = pend; f.hung = hung; }
    void chans(bool i, bool o, int32_t iv, int32_t ov) { f.in_full = i; f.out_full = o; f.in_val = iv; f.out_val = ov; }
    void depth(int s, uint32_t d) { f.depth[s] = d; }
    void entry(int s, uint32_t d, int32_t v) { entries[(size_t)s * cap + d] = v; }
    void call(bool dep, int32_t pin, int pos, bool changed) { f.deposited = dep; f.pin = pin; f.pos = pos; f.changed = changed; }
};
} // namespace

// Session i's state at its hand-off (sess_convert.h).  entries: [stack][cap].
int mkc_sess_export(void *ev, size_t i, orc_flat *f, int32_t *entries)
{
    auto *e = (SessEmu *)ev;
    if (i >= e->sb.size() || e->state[i] != 2) return -1;
    memset(f, 0, sizeof *f);
    const mk::SessMapHdr &h = e->hdr.at(e->hand_sb[i]);
    bool bad = false;
    auto reg = [&](uint32_t r) { return e->R[i].at(r); };
    auto slot = [&](uint32_t s) -> int32_t {
        auto it = e->slots[i].find(s);
        if (it == e->slots[i].end()) { bad = true; return 0; }
        return it->second;
    };
    FlatOut o{*f, entries, e->cap};
    mk::sess_convert(e->N, e->S, h, e->rec.data() + h.off, e->P.dyn_base.data(), reg, slot, o);
    f->entries = entries;
    f->csteps = e->hand_steps[i];
    return bad ? -3 : 0;
}

// The session lane of the native tier (tis_jit.h jit_session_lane) for the
// CPU tests: 0 with the source in `out` and the register / slot counts, 1
// when the compiler declined (why in `out`), negative when `out` is too small.
int mkc_sess_lane(void *hv, uint32_t cap, uint32_t *nregs, uint32_t *nslots, char *out, size_t out_len)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w, src;
    mk::SchedLimits lim;
    int rc = 0;
    if (!mk::compile_session_schedule(h->net, cap, lim, P, w) ||
        !mk::jit_session_lane(P, mk::JitLimits::from_env(), src, w)) {
        src = w;
        rc = 1;
    }
    *nregs = P.nregs;
    *nslots = P.nslots;
    if (src.size() + 1 > out_len) return -1;
    memcpy(out, src.c_str(), src.size() + 1);
    return rc;
}

// The longest call of the session schedule (tis_jit.h
// jit_session_max_call_steps; UINT64_MAX: unbounded): 0, or 1 when the
// session compiler declined.
int mkc_sess_call_steps(void *hv, uint32_t cap, uint64_t *out)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w;
    if (!mk::compile_session_schedule(h->net, cap, mk::SchedLimits{}, P, w)) return 1;
    *out = mk::jit_session_max_call_steps(P, mk::JitLimits::from_env());
    return 0;
}

// The whole session module (lane + mk_sess_exec) as hiprtc gets it.
int mkc_sess_module(void *hv, uint32_t cap, char *out, size_t out_len)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w, src;
    int rc = 0;
    if (!mk::compile_session_schedule(h->net, cap, mk::SchedLimits{}, P, w) ||
        !mk::jit_session_source(P, mk::JitLimits::from_env(), src, w)) {
        src = w;
        rc = 1;
    }
    if (src.size() + 1 > out_len) return -1;
    memcpy(out, src.c_str(), src.size() + 1);
    return rc;
}

// Lane function of the native tier (tis_jit.h) for the CPU tests: returns 0
// with the source in `out`, 1 when the schedule or the JIT declined (why in
// `out`), negative when `out` is too small.
int mkc_jit_lane(void *hv, uint32_t cap, int soo, int force_machine, uint32_t *nslots, int *shape, char *out,
                 size_t out_len)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w, src;
    mk::SchedLimits lim;
    mk::JitLimits jl = mk::JitLimits::from_env();
    jl.force_machine = force_machine != 0;
    if (force_machine) jl.force_stream = false;
    mk::JitShape sh = mk::JIT_STREAM;
    int rc = 0;
    if (!mk::compile_schedule(h->net, cap, soo != 0, lim, P, w) || !mk::jit_lane_source(P, jl, src, w, &sh, nullptr, nullptr, true)) {
        src = w;
        rc = 1;
    }
    *nslots = P.nslots;
    *shape = (int)sh;
    if (src.size() + 1 > out_len) return -1;
    memcpy(out, src.c_str(), src.size() + 1);
    return rc;
}

// The tier a launch with the default budget lands on, decided as the
// product library decides it (mk_exec.hip pick_tier, without hiprtc):
// 3 = native (tis_jit), 2 = compiled schedule (tier 2), 1 = interpreter.
// `why` gets the shape (tier 3) or the reason for falling back.
int mkc_tier(void *hv, uint32_t cap, int soo, char *why, size_t why_len)
{
    auto *h = (CheckNet *)hv;
    mk::SchedProgram P;
    std::string w, src;
    mk::SchedLimits lim;
    int tier = 1;
    if (mk::compile_schedule(h->net, cap, soo != 0, lim, P, w)) {
        const mk::JitLimits jl = mk::JitLimits::from_env();
        mk::JitShape sh = mk::JIT_STREAM;
        bool heavy = false;
        uint32_t pool = 0;
        if (mk::jit_lane_source(P, jl, src, w, &sh, nullptr, &heavy, false, &pool)) {
            tier = 3;
            w = sh == mk::JIT_MACHINE ? (pool ? "machine-pool" : "machine") : heavy ? "stream-heavy" : "stream";
        } else {
            tier = P.nsb > 1024 ? 1 : 2; // mk_exec.hip pick_tier: kSchedInterpSb
        }
    }
    if (why && why_len) {
        const size_t k = std::min(why_len - 1, w.size());
        memcpy(why, w.data(), k);
        why[k] = 0;
    }
    return tier;
}

// The front end alone (tis_front.cpp parse_program), in mk_tokenize's output
// form: token vectors, lines joined by '\n', tokens by '\x1f'; 0 or the
// Go error text with -2 (MK_EPARSE); -3 when `out` is too small.  For the
// sanitized build, which runs the front-end golden vectors through it.
int mkc_tokenize(const char *program, char *out, size_t out_len)
{
    if (!program || !out || !out_len) return -1;
    mk::Program P;
    std::string err, s;
    const bool ok = mk::parse_program(program, P, err);
    if (!ok) {
        s = err;
    } else {
        for (size_t i = 0; i < P.lines.size(); i++) {
            if (i) s += '\n';
            s += mk::form_name(P.lines[i].form);
            if (!P.lines[i].a.empty()) { s += '\x1f'; s += P.lines[i].a; }
            if (!P.lines[i].b.empty()) { s += '\x1f'; s += P.lines[i].b; }
        }
    }
    if (s.size() + 1 > out_len) return -3;
    std::memcpy(out, s.c_str(), s.size() + 1);
    return ok ? 0 : -2;
}

} // extern "C"
