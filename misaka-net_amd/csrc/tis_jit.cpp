// tis_jit.cpp -- code generator of tier 3 (see tis_jit.h).  Host C++ only:
// it produces source text; mk_exec.hip compiles it with hiprtc and the check
// library (sched_check.cpp) exposes the lane function to the CPU tests, which
// compile it with g++ and compare it with the oracle.
//
// The input is the device form of the schedule (assemble_device with 8-byte
// register stride, so register r has operand r*8) -- the same stream the
// tier-2 kernel interprets and the host model in sched_check.cpp executes --
// and each micro-op is restated exactly as those two execute it.
#include "tis_jit.h"

#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <deque>
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
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        s += buf;
        s += '\n';
    }
};

// Operand A/B: register value, sign-extended from its low 32 bits when the
// micro-op says so (UF_TA / UF_TB).
std::string operand(uint32_t off, bool trunc)
{
    char b[64];
    if (trunc)
        snprintf(b, sizeof b, "((int64_t)(int32_t)r%u)", off / 8);
    else
        snprintf(b, sizeof b, "r%u", off / 8);
    return b;
}

std::string u64lit(int64_t v)
{
    char b[32];
    snprintf(b, sizeof b, "0x%016" PRIx64 "ull", (uint64_t)v);
    return b;
}

std::string result(const DOp &I)
{
    if (I.fl & UF_OUTREG) return "(int32_t)" + operand(I.a, I.fl & UF_TA);
    char b[48];
    snprintf(b, sizeof b, "(int32_t)%" PRId32, (int32_t)I.imm);
    return b;
}

} // namespace

bool jit_lane_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why)
{
    std::vector<uint32_t> entry;
    const std::vector<DOp> D = assemble_device(p, 8, entry);
    const size_t nv = entry.size();
    if (nv == 0) {
        why = "empty schedule";
        return false;
    }
    // reachable variants from variant 0 (the entry superblock, fast variant)
    std::vector<char> seen(nv, 0);
    std::deque<uint32_t> work{0};
    seen[0] = 1;
    size_t nreach = 0, ndops = 0;
    std::vector<char> used_reg(p.nregs + 1, 0);
    used_reg[p.in_reg] = 1;
    auto reach = [&](uint64_t v) -> bool {
        if (v >= nv) return false;
        if (!seen[v]) {
            seen[v] = 1;
            work.push_back((uint32_t)v);
        }
        return true;
    };
    while (!work.empty()) {
        const uint32_t v = work.front();
        work.pop_front();
        if (++nreach > lim.max_variants) {
            why = "too many superblock variants for the native tier";
            return false;
        }
        for (size_t pc = entry[v];; ++pc) {
            if (pc >= D.size()) {
                why = "superblock runs off the code";
                return false;
            }
            if (++ndops > lim.max_dops) {
                why = "schedule too large for the native tier";
                return false;
            }
            const DOp &I = D[pc];
            auto use = [&](uint32_t off) {
                if (off / 8 < used_reg.size()) used_reg[off / 8] = 1;
            };
            bool leave = false, ok = true;
            switch (I.op) {
            case U_MOV: case U_ADDI: case U_RSUBI: use(I.a); use(I.d); break;
            case U_ADD: case U_SUB: use(I.a); use(I.b); use(I.d); break;
            case U_LI: case U_LD: use(I.d); break;
            case U_ST: use(I.a); break;
            case U_STI: break;
            case U_JUMP: ok = reach((uint64_t)I.imm); leave = true; break;
            case U_BR:
                use(I.a);
                ok = reach((uint32_t)(uint64_t)I.imm) && reach((uint64_t)I.imm >> 32);
                leave = true;
                break;
            case U_JRO:
                use(I.a);
                for (uint64_t t = 0; t <= I.b && ok; ++t) {
                    const uint64_t j = (uint64_t)I.imm + t;
                    ok = j < p.jtab.size() && reach(p.jtab[j]);
                }
                leave = true;
                break;
            case U_END: if (I.fl & UF_OUTREG) use(I.a); leave = true; break;
            case U_GUARD: ok = reach((uint64_t)I.imm); break;
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
    for (uint32_t r = 0; r < used_reg.size(); ++r)
        if (used_reg[r] && r >= p.nregs) {
            why = "register out of range";
            return false;
        }

    Emitter e;
    e.line("// generated from a compiled schedule: %zu variants reachable, %zu micro-ops", nreach, ndops);
    e.line("MK_FN int32_t mk_lane(int64_t in, uint32_t budget, int32_t *__restrict__ slots, uint64_t sstride,");
    e.line("                      uint32_t *steps_out, uint32_t *status_out)");
    e.line("{");
    for (uint32_t r = 0; r < p.nregs; ++r)
        if (used_reg[r]) e.line("    int64_t r%u = 0;", r);
    e.line("    r%u = (int64_t)(int32_t)in;", p.in_reg);
    e.line("    uint32_t steps = 0, st = 0;");
    e.line("    int32_t outv = 0;");
    e.line("    (void)slots; (void)sstride; (void)budget;");
    for (uint32_t v = 0; v < nv; ++v) {
        if (!seen[v]) continue;
        e.line("V%u:", v);
        for (size_t pc = entry[v];; ++pc) {
            const DOp &I = D[pc];
            const bool ta = I.fl & UF_TA, tb = I.fl & UF_TB;
            const std::string A = operand(I.a, ta), B = operand(I.b, tb);
            const uint32_t d = I.d / 8;
            bool leave = false;
            switch (I.op) {
            case U_MOV: e.line("    r%u = %s;", d, A.c_str()); break;
            case U_LI: e.line("    r%u = (int64_t)%s;", d, u64lit(I.imm).c_str()); break;
            case U_ADD: e.line("    r%u = (int64_t)((uint64_t)%s + (uint64_t)%s);", d, A.c_str(), B.c_str()); break;
            case U_SUB: e.line("    r%u = (int64_t)((uint64_t)%s - (uint64_t)%s);", d, A.c_str(), B.c_str()); break;
            case U_ADDI: e.line("    r%u = (int64_t)((uint64_t)%s + %s);", d, A.c_str(), u64lit(I.imm).c_str()); break;
            case U_RSUBI: e.line("    r%u = (int64_t)(%s - (uint64_t)%s);", d, u64lit(I.imm).c_str(), A.c_str()); break;
            case U_ST:
                e.line("    slots[(uint64_t)%uu * sstride] = (int32_t)%s;", (uint32_t)I.imm, A.c_str());
                break;
            case U_STI:
                e.line("    slots[(uint64_t)%uu * sstride] = (int32_t)%" PRId32 ";", I.d, (int32_t)I.imm);
                break;
            case U_LD: e.line("    r%u = (int64_t)slots[(uint64_t)%uu * sstride];", d, (uint32_t)I.imm); break;
            case U_JUMP:
                e.line("    steps += %uu;", I.inc);
                e.line("    goto V%u;", (uint32_t)I.imm);
                leave = true;
                break;
            case U_BR: {
                static const char *const cmp[4] = {"== 0", "!= 0", "> 0", "< 0"};
                const uint32_t c = (I.fl >> UF_COND_SHIFT) & 3u;
                e.line("    steps += %uu;", I.inc);
                e.line("    if (%s %s) goto V%u;", A.c_str(), cmp[c], (uint32_t)(uint64_t)I.imm);
                e.line("    goto V%u;", (uint32_t)((uint64_t)I.imm >> 32));
                leave = true;
                break;
            }
            case U_JRO: {
                // IntClamp(ip + A, 0, len-1) with an int64 wrapping add (program.go:354,362)
                e.line("    steps += %uu;", I.inc);
                e.line("    {");
                e.line("        int64_t t = (int64_t)((uint64_t)%uu + (uint64_t)%s);", I.d, A.c_str());
                e.line("        t = t > (int64_t)%u ? (int64_t)%u : t;", I.b, I.b);
                e.line("        t = t < 0 ? 0 : t;");
                e.line("        switch (t) {");
                const uint32_t last = p.jtab[(size_t)I.imm + I.b];
                for (uint32_t t = 0; t < I.b; ++t) {
                    const uint32_t tgt = p.jtab[(size_t)I.imm + t];
                    if (tgt != last) e.line("        case %u: goto V%u;", t, tgt);
                }
                e.line("        default: goto V%u;", last);
                e.line("        }");
                e.line("    }");
                leave = true;
                break;
            }
            case U_END:
                e.line("    steps += %uu;", I.inc);
                e.line("    outv = %s;", result(I).c_str());
                e.line("    st = %uu;", I.d);
                e.line("    goto done;");
                leave = true;
                break;
            case U_GUARD:
                e.line("    if ((uint64_t)steps + %uu >= (uint64_t)budget) goto V%u;", I.inc, (uint32_t)I.imm);
                break;
            case U_ROUND_END:
                e.line("    if ((uint64_t)steps + %uu >= (uint64_t)budget) {", I.inc);
                e.line("        steps += %uu;", I.inc);
                e.line("        outv = %s;", result(I).c_str());
                e.line("        st = %uu;", I.d);
                e.line("        goto done;");
                e.line("    }");
                break;
            }
            if (leave) break;
        }
    }
    e.line("done:");
    e.line("    *steps_out = steps;");
    e.line("    *status_out = st;");
    e.line("    return outv;");
    e.line("}");
    src = std::move(e.s);
    return true;
}

std::string jit_module_source(const std::string &lane_src)
{
    Emitter e;
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
    e.s += kDeviceCommon;
    e.s += "\n";
    e.s += lane_src;
    // One lane per thread per iteration, grid-stride over the batch; the next
    // input is loaded before the current lane runs, so its HBM latency hides
    // behind the lane's work.  Counters fold per wave (stats_reduce).
    e.s += R"(
extern "C" __global__ void __launch_bounds__(256) mk_jit_exec(SParams p)
{
    const uint64_t gid = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
    int32_t *slots = p.slots ? p.slots + gid : (int32_t *)0;
    uint64_t i = gid;
    int32_t cur = i < p.n ? sched_input(p, i) : 0;
    for (; i < p.n; i += stride) {
        const int32_t nxt = i + stride < p.n ? sched_input(p, i + stride) : 0;
        uint32_t steps, st;
        const int32_t o = mk_lane(cur, p.budget, slots, p.lanes, &steps, &st);
        p.out[i] = (st & MK_ST_HAS_OUTPUT) ? o : 0;
        p.status[i] = (uint8_t)st;
        if (p.steps) p.steps[i] = steps;
        count_lane(cnt, steps, st);
        cur = nxt;
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}
)";
    return e.s;
}

} // namespace mk
