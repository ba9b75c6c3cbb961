/*
 * mk.h -- C ABI of the MI355X batched executor for Misaka Net TIS networks.
 *
 * Drop-in boundary (SURVEY.md section 8 row b).  The reference has no FFI; the
 * path sits behind the master's HTTP surface and the Go-internal node types.
 * Each entry point below names the reference interface it replaces.  Plain C:
 * no C++ types, caller-owned arrays, the library never retains a caller
 * pointer after return (cgo pointer-passing rules), never exits or aborts.
 *
 * Thread safety: every call is safe to make concurrently on one mk_net
 * (Go net/http runs /compute handlers concurrently, master.go:197).  The host
 * API serialises per handle.  Launches of one handle on one device share its
 * scratch (stack slots, counters), so the library orders them across
 * streams: work enqueued on a stream other than the previous launch's waits
 * for that launch (the host API's internal stream included).  Callers that
 * never change stream pay nothing for it.
 */
#ifndef MK_H
#define MK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (negative returns) ---------------------------------- */
#define MK_OK 0
#define MK_EINVAL (-1)  /* bad argument                                   */
#define MK_EPARSE (-2)  /* program text rejected (Go error text in err)   */
#define MK_ELIMIT (-3)  /* network exceeds executor limits                */
#define MK_EDEVICE (-4) /* HIP runtime error / no usable GPU              */
#define MK_ENOMEM (-5)  /* allocation failed                              */
#define MK_EBUSY (-6)   /* would block: port full / stack empty (retry)  */

/* ---- limits ------------------------------------------------------------ */
#define MK_MAX_PROGRAM_NODES 16
#define MK_MAX_STACK_NODES 32
#define MK_MAX_LINES 65535

/* ---- per-lane status byte ---------------------------------------------- */
#define MK_ST_QUIESCENT 1      /* every node blocked (reference: /compute hangs if no output) */
#define MK_ST_BUDGET 2         /* retired-instruction budget reached at a round end           */
#define MK_ST_STACK_OVERFLOW 3 /* a PUSH exceeded stack_cap (reference stacks are unbounded)  */
#define MK_ST_OUTPUT_STOP 4    /* stopped at the first OUT (MK_FLAG_STOP_ON_OUTPUT)           */
#define MK_ST_REMOTE_WAIT 5    /* session call parked on remote peers / inbound RPCs (row f4)  */
#define MK_ST_CALL_OPEN 6      /* session: a call is still open; this new one did nothing      */
#define MK_ST_REASON_MASK 0x0f
#define MK_ST_HAS_OUTPUT 0x10  /* lane produced a /compute result                              */

/* ---- node kinds ----------------------------------------------------------
 * NODE_INFO types (master.go:431-438, docker-compose.yml:16-21) plus the
 * master's own name (MASTER_URI, cmd/app.go:20): a program that addresses the
 * master with MOV/PUSH/POP gets the reference's Unimplemented-and-retry
 * behaviour instead of the unknown-host hang. */
#define MK_NODE_PROGRAM 0
#define MK_NODE_STACK 1
#define MK_NODE_MASTER 2
/* Peers served outside this executor -- reference nodes of a mixed
 * deployment (row f4): MOV to a remote program's port, PUSH / POP on a
 * remote stack become requests a stateful session hands to its host, which
 * makes the reference's RPC (Program.Send, Stack.Push / Stack.Pop,
 * messenger.proto:9-28; see mk_session_remote_*).  Batch lanes have no
 * peers: such an instruction blocks there forever. */
#define MK_NODE_REMOTE_PROGRAM 3
#define MK_NODE_REMOTE_STACK 4

typedef struct mk_net mk_net;

typedef struct {
    const char *name;    /* service name other nodes address it by          */
    int kind;            /* MK_NODE_*                                        */
    const char *program; /* TIS source for MK_NODE_PROGRAM (NULL = "")     */
} mk_node_desc;

#define MK_FLAG_STOP_ON_OUTPUT 1u
/* Skip the schedule compiler and run the direct bytecode interpreter
 * (tier 1).  By default a network is first compiled into superblocks of
 * micro-ops (tier 2); networks the compiler cannot bound fall back to
 * tier 1 automatically.  Both tiers give identical results. */
#define MK_FLAG_FORCE_INTERP 2u
/* Select the tier-2 superblock interpreter with the given lane scheduling
 * (results are identical either way; tier 2's default is TILE).  TILE: every
 * thread owns K contiguous inputs of a tile and the tile is written back with
 * vector stores once all of its lanes finished.  REFILL: a finished slot
 * immediately takes the next input. */
#define MK_FLAG_TILE 4u
#define MK_FLAG_REFILL 8u
/* Tier 3: the compiled schedule as a native gfx950 kernel generated and
 * compiled (hiprtc) once per network and option set.  Used by default when
 * the schedule fits its limits; MK_FLAG_JIT demands it (MK_ELIMIT when it is
 * unavailable -- mk_net_plan gives the reason), MK_FLAG_TILE / MK_FLAG_REFILL
 * select the tier-2 superblock interpreter, MK_FLAG_FORCE_INTERP tier 1.
 * MK_JIT=0 in the environment disables tier 3. */
#define MK_FLAG_JIT 16u
/* Device API: gather the counters of this launch without folding them into
 * d_stats yet (d_stats may be NULL).  Counters of deferred launches on one
 * handle and device accumulate on the device until mk_stats_fold (or the
 * next launch that folds); launches that defer must be stream-ordered with
 * each other and with the fold. */
#define MK_FLAG_DEFER_STATS 32u

typedef struct {
    uint32_t budget;      /* retired node-instructions per lane; 0 = 1<<20          */
    uint32_t stack_cap;   /* values per stack per lane; 0 = 1024                     */
    uint32_t flags;       /* MK_FLAG_*                                               */
    uint32_t device_mask; /* host API: GPUs to shard the batch over; 0 = GPU 0 only */
} mk_opts;

/* Parse + lower every program node and wire ports/stacks.
 * Replaces: ProgramNode.LoadProgram (internal/nodes/program.go:178-193) ->
 * tis.GenerateLabelMap / tis.Tokenize (internal/tis/tokenizer.go:11-106) for
 * every node of NODE_INFO (cmd/app.go:31), plus the name resolution that the
 * reference does per call with grpc.Dial (program.go:492,510,525).
 * Parse errors return MK_EPARSE with "node <name>: <Go error text>" in err,
 * where the Go text is byte-identical to the reference's
 * ("Cannot repeat label", "line N, label 'L' was not declared",
 *  "line N, '<instr>' not a valid instruction"). */
int mk_net_load(const mk_node_desc *nodes, int n, mk_net **out, char *err, size_t err_len);

void mk_net_free(mk_net *net);

/* Evaluate n independent /compute inputs (host arrays).
 * Replaces: the /compute handler (master.go:197-224) + GetInput/SendOutput
 * (master.go:233-249) + the program/stack node loops (program.go:80-92,
 * stack.go:95-155) for a batch.  in[i] is the strconv.Atoi value of the form
 * field; it is truncated to int32 inside, as GetInput does (master.go:237).
 * out[i] is the first OUT value (what /compute returns), status[i] the
 * MK_ST_* byte, steps[i] (nullable) the retired node-instructions. */
int mk_compute_batch(mk_net *net, const int64_t *in, size_t n, int32_t *out, uint8_t *status,
                     uint32_t *steps, const mk_opts *opts);

/* ---- device API (inputs/outputs already in HBM) ------------------------- */
#define MK_IN_I64 0 /* data: const int64_t*                                   */
#define MK_IN_I32 1 /* data: const int32_t*                                   */
#define MK_IN_GEN 2 /* synthetic: x_i = gen(seed, offset + i), no input bytes */

#define MK_GEN_FULL 0   /* (int32)splitmix64(seed^i); lanes i%16==15 take int32 edge values */
#define MK_GEN_MASKED 1 /* splitmix64(seed^i) & mask                                          */

typedef struct {
    int kind;          /* MK_IN_*                               */
    const void *data;  /* device pointer (MK_IN_I64 / MK_IN_I32) */
    uint64_t seed;     /* MK_IN_GEN                             */
    uint32_t gen_kind; /* MK_GEN_*                              */
    uint32_t gen_mask;
    uint64_t offset;   /* global lane index of element 0        */
} mk_input;

/* stats (nullable, device uint64[8], accumulated, caller zeroes):
 * [0] retired node-instructions  [1] lanes with output  [2] lanes finished
 * [3] quiescent  [4] budget  [5] stack overflow  [6] output-stop  [7] reserved */
#define MK_STATS_LEN 8

/* Launch the executor on `device` on HIP stream `stream` (NULL = default).
 * d_out / d_status are required, d_steps / d_stats nullable.  Asynchronous. */
int mk_compute_device(mk_net *net, int device, const mk_input *in, size_t n, int32_t *d_out,
                      uint8_t *d_status, uint32_t *d_steps, uint64_t *d_stats,
                      const mk_opts *opts, void *stream);

/* ---- stateful sessions ------------------------
 * The reference's nodes keep running between /compute calls
 * (program.go:80-92): ACC, BAK, ptr, ports, stacks and the master's inChan /
 * outChan (capacity 1, master.go:58-59) persist from one call to the next.
 * A session set holds n such network instances in HBM, in the post-/reset,
 * post-/run state; one compute call performs one /compute (master.go:
 * 216-219) on every session at once: deposit in[i] once inChan is empty,
 * run until outChan holds a value and take it.  status[i] is
 * MK_ST_HAS_OUTPUT with out[i] the value, or why the call has no result:
 *   MK_ST_BUDGET: this slice of the call retired opts->budget instructions.
 *     The call stays OPEN -- the reference's handler keeps waiting while its
 *     nodes run on (program.go:80-92) -- and mk_session_step(in = NULL)
 *     continues it with a fresh budget; mk_session_cancel abandons it.
 *   MK_ST_QUIESCENT: nothing can change without another input (the
 *     reference's handler would block forever).  The call closes; the
 *     instance keeps its state and takes the next call's input.
 *   MK_ST_STACK_OVERFLOW: a PUSH beyond stack_cap (the reference's stacks
 *     are unbounded): the session stays ended (same status, no output) until
 *     mk_session_reset.
 *   MK_ST_CALL_OPEN: the session already had an open call; this call did
 *     nothing and its input was not taken.  The host calls return MK_EBUSY
 *     when any session had a call open as the launch began (a burst's later
 *     calls behind a call that stayed open in the same launch report it too,
 *     without MK_EBUSY).
 * steps[i] (nullable): instructions retired by the call so far, over all
 * its slices (mod 2^32).  The mk_net must outlive its sessions. */
typedef struct mk_session mk_session;

int mk_session_create(mk_net *net, int device, size_t n, const mk_opts *opts, mk_session **out);

/* One /compute call on every session (host arrays; synchronous). */
int mk_session_compute(mk_session *s, const int64_t *in, int32_t *out, uint8_t *status, uint32_t *steps);

/* ncalls sequential /compute calls on every session in one launch (host
 * arrays laid out [call][session]; synchronous): call c of session i takes
 * in[c*n + i] and reports out/status/steps[c*n + i], exactly as ncalls
 * mk_session_compute calls in a row would.  Replaces a burst of concurrent
 * /compute requests on the reference's one network (master.go:197-224 served
 * one at a time through inChan/outChan, :216-219); the master coalesces such
 * bursts into one call (misaka_net_amd.master). */
int mk_session_compute_seq(mk_session *s, const int64_t *in, size_t ncalls, int32_t *out, uint8_t *status,
                           uint32_t *steps);

/* One call on device arrays, asynchronous on `stream` (NULL = the session's
 * own stream); calls on one session are ordered device-side, with no host
 * synchronisation: a call waits on an event recorded after the previous
 * launch when that ran on another stream (calls on one stream follow stream
 * order), and the session's synchronous calls below wait on it too.  The
 * event is the completion event of the launch's last kernel (no separate
 * marker on the stream: ~3 us per call less).  A
 * caller stream must outlive the session work queued on it; mk_session_free
 * waits for the last launch on any stream. */
int mk_session_compute_device(mk_session *s, const int64_t *d_in, int32_t *d_out, uint8_t *d_status,
                              uint32_t *d_steps, void *stream);

/* mk_session_compute_seq on device arrays ([call][session], d_steps
 * nullable), asynchronous on `stream` like mk_session_compute_device: a burst
 * of ncalls sequential /compute calls per instance in one launch, the state
 * loaded from HBM once and stored once.  Statuses report MK_ST_CALL_OPEN as
 * the host call does; nothing here returns MK_EBUSY (the statuses stay on the
 * device). */
int mk_session_compute_seq_device(mk_session *s, const int64_t *d_in, size_t ncalls, int32_t *d_out,
                                  uint8_t *d_status, uint32_t *d_steps, void *stream);

/* ---- mixed deployments (row f4): sessions of a network with remote peers --
 * A call on such a session runs until it has its output or nothing more can
 * happen without the peers; then it is PARKED: status MK_ST_REMOTE_WAIT,
 * no output, the call still open.  The host then
 *   - makes the RPC of every outstanding request (mk_session_remote_poll:
 *     Program.Send to a remote port, Stack.Push / Stack.Pop on a remote stack,
 *     program.go:475-536) and reports each completion (mk_session_remote_done,
 *     with the popped value for a pop);
 *   - serves the peers' RPCs to this instance's nodes: Program.Send into a
 *     local port (mk_session_port_put, MK_EBUSY while full: program.go:163),
 *     Stack.Push / Stack.Pop on a local stack (mk_session_stack_push / _pop,
 *     MK_EBUSY while empty: stack.go:133-155), and Master.GetInput /
 *     SendOutput on the master's channels (mk_session_input_take /
 *     _output_put);
 *   - resumes the call (mk_session_step with in = NULL).
 * All of these are ordered on the session's stream and synchronous. */
#define MK_REMOTE_SEND 0
#define MK_REMOTE_PUSH 1
#define MK_REMOTE_POP 2
typedef struct {
    uint32_t node;   /* local program node (sorted-name index) making the request */
    uint32_t op;     /* MK_REMOTE_*                                              */
    uint32_t remote; /* index of the peer among the network's MK_NODE_REMOTE_* nodes */
    uint32_t reg;    /* MK_REMOTE_SEND: the peer's port R0..R3                   */
    int32_t value;   /* SEND / PUSH: int32 value                                 */
} mk_remote_req;

/* One call step on every session: a new /compute call with in[i] (host
 * arrays), or, with in == NULL, resume each session's open call (parked on
 * peers, or out of budget); sessions without one report status 0. */
int mk_session_step(mk_session *s, const int64_t *in, int32_t *out, uint8_t *status, uint32_t *steps);
int mk_session_remote_poll(mk_session *s, size_t inst, mk_remote_req *reqs, int max, int *count);
int mk_session_remote_done(mk_session *s, size_t inst, uint32_t node, int32_t value);
int mk_session_port_put(mk_session *s, size_t inst, uint32_t node, uint32_t reg, int32_t value);
int mk_session_stack_push(mk_session *s, size_t inst, uint32_t stack, int32_t value);
int mk_session_stack_pop(mk_session *s, size_t inst, uint32_t stack, int32_t *value);
/* The master's side for remote program nodes that do IN / OUT: their
 * Master.GetInput takes from this instance's inChan (master.go:233-242;
 * MK_EBUSY while it is empty and no open call holds an input to deposit --
 * the reference's receive blocks), their Master.SendOutput deposits into its
 * outChan (master.go:245-249; MK_EBUSY while full).  The open call takes
 * that output when it resumes. */
int mk_session_input_take(mk_session *s, size_t inst, int32_t *value);
int mk_session_output_put(mk_session *s, size_t inst, int32_t value);

/* Kind (MK_NODE_*) and index of a node by name: program and stack nodes in
 * sorted-name order (the canonical schedule), remote peers in declaration
 * order. */
int mk_net_node_index(const mk_net *net, const char *name, int *kind, int *index);

/* Abandon every session's open call (the master answered it 504).  What it
 * set in motion stays: an input it deposited in inChan, the nodes' progress;
 * an input not deposited yet is dropped.  Synchronous. */
int mk_session_cancel(mk_session *s);

/* Which tier runs the sessions, as one line of text: "tier=native ..." --
 * the network's session schedule compiled to a kernel (one thread per
 * session, state in HBM; a call whose budget slice ends inside a superblock
 * is handed to the interpreter, which keeps that session) -- or
 * "tier=interp reason=..." (the bytecode interpreter for every session:
 * mixed deployments, networks the compiler declines, MK_SESSION_NATIVE=0).
 * Host-side state access (mk_session_port_put, _stack_*, _input_take,
 * _output_put) is for interpreter sessions: MK_EINVAL on the native tier. */
int mk_session_plan(const mk_session *s, char *out, size_t out_len);

/* /reset (master.go:126-143): every session back to the initial state. */
int mk_session_reset(mk_session *s);

void mk_session_free(mk_session *s);

/* Add the counters accumulated by MK_FLAG_DEFER_STATS launches on `device`
 * into d_stats (device uint64[MK_STATS_LEN]) and clear them; asynchronous
 * on `stream`.  Replaces nothing in the reference (it has no counters). */
int mk_stats_fold(mk_net *net, int device, uint64_t *d_stats, void *stream);

/* Fill d_out[i] = gen(seed, offset + i) on device (same generator as MK_IN_GEN). */
int mk_generate_inputs_device(int device, uint64_t seed, uint32_t gen_kind, uint32_t gen_mask,
                              uint64_t offset, size_t n, int32_t *d_out, void *stream);

/* ---- lane trace -------------------------------------
 * The reference logs every instruction it executes (log.Printf of tokens,
 * ACC, BAK; program.go:222-223).  mk_trace_lane runs ONE /compute input
 * through the bytecode interpreter (tier 1, the tier that executes one TIS
 * instruction at a time) on `device` and returns its first max_entries
 * retired instructions in schedule order: round, program node (index in
 * sorted-name order), the ptr it executed at, ACC and BAK after it -- the
 * same records as the oracle's orc_trace_lane, so a lane whose result
 * differs can be diffed instruction by instruction.  *count = entries
 * written, *status = the lane's MK_ST_* byte.  Synchronous. */
typedef struct {
    uint32_t round;
    uint16_t node;
    uint16_t ip;
    int64_t acc;
    int64_t bak;
} mk_trace_entry;

int mk_trace_lane(mk_net *net, int device, int64_t input, const mk_opts *opts, mk_trace_entry *out,
                  uint32_t max_entries, uint32_t *count, uint8_t *status);

/* ---- introspection -------------------------------------------------------- */
/* Token dump of one program in the test format: lines joined by '\n', tokens
 * by '\x1f' (the [][]string of tis.Tokenize); on error the Go error text and
 * MK_EPARSE.  Replaces tis.Tokenize for parity tests. */
int mk_tokenize(const char *program, char *out, size_t out_len);

/* Lowered bytecode of a loaded network as text (one instruction per line). */
int mk_net_disasm(const mk_net *net, char *out, size_t out_len);

/* Which tier `opts` selects for this network and its shape, as one line of
 * text ("tier=native ..", "tier=compiled superblocks=.. regs=.. words=.." or
 * "tier=interp reason=.."); compiles the schedule (and the native kernel) if
 * not cached yet. */
int mk_net_plan(mk_net *net, const mk_opts *opts, char *out, size_t out_len);

/* Compile everything `opts` will use on `device` now (schedule, native
 * kernel, device tables) so the first mk_compute_* call does not pay for it.
 * Replaces nothing in the reference (its /load has no compile step); meant
 * for the master's /load and for benchmarks. */
int mk_net_prepare(mk_net *net, const mk_opts *opts, int device);

/* Generated source of the native (tier-3) kernel for `opts` (MK_ELIMIT with
 * the reason in `out` when the tier is unavailable). */
int mk_net_jit_source(mk_net *net, const mk_opts *opts, char *out, size_t out_len);

/* Micro-op listing of the compiled schedule for `opts` (MK_ELIMIT if the
 * network is not compilable). */
int mk_net_sched_disasm(mk_net *net, const mk_opts *opts, char *out, size_t out_len);

/* counts: [0] program nodes [1] stack nodes [2] total instructions */
int mk_net_info(const mk_net *net, int *counts3);

/* Integer-issue peak probe: launches a dependency-free v_add_u32 kernel doing
 * `iters` x 64 adds per lane over blocks x 256 lanes; returns the lane-op count
 * it performs in *lane_ops.  Caller times it with events on `stream`. */
int mk_valu_probe_device(int device, int blocks, int iters, uint64_t *lane_ops, void *stream);

const char *mk_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MK_H */
