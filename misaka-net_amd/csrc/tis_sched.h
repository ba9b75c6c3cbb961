// tis_sched.h -- schedule compiler: lowers a network's canonical schedule
// (SURVEY.md section 8.0 lane model) into "superblocks" of data micro-ops.
//
// Control state (instruction pointers, port full bits, pending sends, stack
// depths, IN/OUT counters) only depends on data at JEZ/JNZ/JGZ/JLZ/JRO whose
// operand is not a compile-time constant.  The compiler executes the
// schedule symbolically on the host; every blocked attempt, every jump on a
// constant, every register move, SWP, port hand-off and stack push/pop whose
// value stays in a register costs nothing at run time.  What remains is a
// short stream of int64 micro-ops per superblock, ending in a per-lane exit
// (branch on data, multiway JRO, jump to a merged state, or END).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "tis_front.h"

namespace mk {

enum UOpCode : uint8_t {
    U_MOV = 0,  // R[d] = A
    U_LI,       // R[d] = imm
    U_ADD,      // R[d] = A + B
    U_SUB,      // R[d] = A - B
    U_ADDI,     // R[d] = A + imm
    U_RSUBI,    // R[d] = imm - A
    U_ST,       // slot[imm] = int32(A)
    U_STI,      // slot[a]   = int32(imm)
    U_LD,       // R[d] = sext32(slot[imm])
    U_STX,      // slot[imm + R[b]] = int32(A)       (dynamic stack: R[b] = depth)
    U_LDX,      // R[d] = sext32(slot[imm + R[b]])
    U_JUMP,     // steps += d | a<<16; sb = imm                                  (1 word)
    U_BR,       // steps += ext.imm; sb = cond(A) ? lo32(imm) : hi32(imm)         (2 words)
    U_JRO,      // steps += ext.imm; sb = jtab[imm + clamp(d + A, 0, b)]          (2 words)
    U_END,      // steps += ext.imm; out = OUTREG ? A : imm; status = d           (2 words)
    U_GUARD,    // if steps + (d | a<<16) >= budget: sb = imm (checked variant)   (1 word)
    U_ROUND_END,// if steps + ext.imm >= budget: END(status d, out A|imm)          (2 words)
    U_OVF,      // if R[b] >= hi32(ext.imm): steps += lo32(ext.imm); END(status d, out A|imm)
                // (a PUSH onto a dynamic stack at its capacity)                 (2 words)
    U_BRX,      // if cond(A): steps += ext.imm; sb = imm (an in-line side exit)  (2 words)
    // sessions (compile_session_schedule) only:
    U_YIELD,    // a /compute call ends: steps += lo32(ext.imm); out = OUTREG ? A : hi32(ext.imm);
                // status = d; the session's next call starts at variant imm        (2 words)
    U_HANDOFF,  // the budget slice ends inside this superblock: the lane leaves at the
                // entry of variant imm (its state: SchedProgram::smap) for the
                // bytecode interpreter, which runs the rest of the call      (1 word)
    U_COUNT
};

constexpr uint8_t U_DATA_LAST = U_LDX; // ops <= this are data micro-ops
// ops that may stand inside a superblock's body (data ops and in-line ends)
inline bool body_op(uint32_t op) { return op <= U_DATA_LAST || op == U_ROUND_END || op == U_OVF || op == U_BRX; }

// A = R[a] (sign-extended low 32 bits when UF_TA), B likewise with UF_TB.
enum : uint8_t { UF_TA = 1, UF_TB = 2, UF_OUTREG = 4 };
// U_BR condition in fl bits 4..5: 0 = EZ, 1 = NZ, 2 = GZ, 3 = LZ
constexpr int UF_COND_SHIFT = 4;

struct UOp {
    uint8_t op;
    uint8_t fl;
    uint16_t d;
    uint16_t a;
    uint16_t b;
    int64_t imm;
};
static_assert(sizeof(UOp) == 16, "UOp must be 16 bytes");

struct SchedLimits {
    uint32_t max_superblocks = 16384;
    uint32_t max_uops = 1u << 21;          // total words
    uint32_t max_sb_uops = 1u << 17;       // words per superblock before generalising
    uint32_t max_regs = 96;                // LDS registers per lane
    uint32_t soft_regs = 24;               // above this, spill stack entries to HBM first
    uint32_t idle_rounds = 64;             // rounds without emitted code before generalising
    uint64_t max_rounds = 1ull << 22;      // symbolic rounds in total (compile-time bound)
    uint32_t dyn_depths = 24;              // distinct entry depths before a stack turns dynamic (0 = never)
    uint32_t widen_after = 2;              // states of one shape with other constants before widening (0 = never)
    bool share_slots = true;               // acyclic graphs: stacks never in use together share slots
};

// Stateful sessions (row f2): the state at a superblock entry, as the
// bytecode interpreter's session state needs it (a lane handed off there,
// U_HANDOFF).  Locations are those of the compiler (tis_sched.cpp): ACC(n),
// BAK(n), PORT(4n+k), PENDV(n), INL, OUTL, DEP(s), CIN; each is dead, a
// constant, or in register r.  Stack entries are constants or in slot r.
struct SessSrc {
    uint8_t kind = 0; // 0 dead, 1 constant c, 2 register r, 3 slot r
    uint32_t r = 0;
    int64_t c = 0;
};
struct SessEntry {
    std::vector<uint16_t> ip;
    uint32_t pend = 0, hung = 0;
    uint64_t pfull = 0;
    bool in_avail = false, out_full = false, deposited = false;
    uint8_t pos = 0;      // the next program node to attempt in the current round
    bool changed = false; // something changed earlier in that round
    bool pre = false;     // the call's round-start checks are still to run
    std::vector<SessSrc> loc;              // every location, in the compiler's order
    std::vector<std::vector<SessSrc>> stk; // ordinary stacks: their entries, bottom first
};

// Device form of the session state map (SchedProgram::smap), one header per
// superblock and 16-byte records: at `off`, the nprog instruction pointers
// (constants), then every location in the compiler's order (ACC(n), BAK(n),
// PORT(q), PENDV(n), INL, OUTL, DEP(s), CIN), then per stack a count (a
// constant; 0 for dynamic stacks, whose entries are slots base + j below
// DEP) followed by that many entries.  Read by sess_convert.h.
struct SessSrcDev {
    int64_t c;     // constant
    uint32_t r;    // register or slot
    uint32_t kind; // SessSrc::kind
};
static_assert(sizeof(SessSrcDev) == 16, "SessSrcDev must be 16 bytes");
struct SessMapHdr {
    uint32_t off;   // first record
    uint32_t pend, hung;
    uint32_t flags; // in_avail | out_full << 1 | deposited << 2 | changed << 3 | pre << 4 | pos << 8
    uint64_t pfull;
};
static_assert(sizeof(SessMapHdr) == 24, "SessMapHdr must be 24 bytes");

struct SchedProgram;
void build_sess_map(const SchedProgram &p, int nprog, int nstack, std::vector<SessMapHdr> &hdr,
                    std::vector<SessSrcDev> &rec);

struct SchedProgram {
    std::vector<UOp> code;
    std::vector<uint32_t> entry; // variant id -> first word; 2k = fast, 2k+1 = budget-checked
    std::vector<uint32_t> jtab;  // JRO successor tables (variant ids)
    uint32_t nregs = 0;          // 64-bit registers per lane (LDS)
    uint32_t nslots = 0;         // stack memory slots per lane (HBM, lane-major)
    uint32_t ndyn = 0;           // dynamic stacks (slots [k*cap, (k+1)*cap) each)
    uint32_t in_reg = 0;         // register holding the lane input at entry
    uint32_t nsb = 0;            // superblocks
    uint64_t sym_rounds = 0;     // rounds executed symbolically
    // sessions: every superblock's entry state (U_HANDOFF), the dynamic
    // stacks' first slots (-1: ordinary), the location count
    bool session = false;
    std::vector<SessEntry> smap;
    std::vector<int64_t> dyn_base;
    uint32_t nloc = 0;
};

// Device form of a micro-op (32 bytes = one s_load_dwordx8): every field is
// pre-decoded into its own dword and register operands are LDS byte offsets
// (reg * stride) for the layout the launch uses, so the kernel spends
// no scalar instructions on decoding.  Two-word ops fold their extension
// into `inc`.
//   MOV/ADD/SUB/ADDI/RSUBI/LD/LI: d = dst offset, a/b = src offsets
//   ST: a = src offset, imm = slot      STI: d = slot, imm = value
//   JUMP: inc = steps, imm = target     GUARD: inc = max steps to a round end, imm = checked id
//   BR: a = cond offset, imm = lo:taken hi:not-taken, inc = steps
//   JRO: d = ip, a = operand offset, b = len-1, imm = jtab offset, inc = steps
//   END/ROUND_END: d = status, a = out offset (UF_OUTREG) else imm, inc = steps
//   STX: a = src offset, b = index offset, imm = base slot   LDX: d, b, imm likewise
//   OVF: d = status, a = out offset (UF_OUTREG), b = depth offset, inc = steps,
//        imm = (uint32_t)out value | (uint64_t)limit << 32
//   BRX: a = cond offset (fl bits 4..5 as BR), imm = target variant, inc = steps
struct DOp {
    uint32_t op, fl, d, a, b, inc;
    int64_t imm;
};
static_assert(sizeof(DOp) == 32, "DOp must be 32 bytes");

// Assemble `p` with register operands scaled to `reg_bytes` (the byte stride
// between consecutive registers in the executor's LDS layout).  entry_out[v]
// = first DOp of superblock variant v.
std::vector<DOp> assemble_device(const SchedProgram &p, uint32_t reg_bytes, std::vector<uint32_t> &entry_out);

// Compile for the given stack capacity / stop-on-output option (both change
// the control flow).  Returns false with a reason when a limit is exceeded;
// the caller then uses the direct bytecode interpreter.
bool compile_schedule(const Network &net, uint32_t stack_cap, bool stop_on_output, const SchedLimits &lim,
                      SchedProgram &out, std::string &why);

// The same network compiled for stateful sessions (SURVEY.md section 8 row
// f2; oracle session_step): variant 0 is the post-/reset instance at the
// start of a /compute call whose input is in register in_reg.  A call ends
// in U_YIELD (its output taken, or a round without change: the next call
// starts at the yield's variant, again with its input in in_reg) or U_END
// (a stack overflow ends the session).  Budget-checked variants are a
// U_HANDOFF each: the rest of such a call runs on the interpreter.
bool compile_session_schedule(const Network &net, uint32_t stack_cap, const SchedLimits &lim, SchedProgram &out,
                              std::string &why);

std::string sched_disasm(const SchedProgram &p);

} // namespace mk
