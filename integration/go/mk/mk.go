// Package mk binds the MI355X executor's C ABI (include/mk.h) for the
// reference's Go tree (SURVEY.md section 8 row f3).  A maintainer vendors
// this package next to internal/nodes and selects it in cmd/app.go (see
// INTEGRATION.md).  The Go toolchain is absent from the image this package
// was written in, so it is shipped as source: not compiled or tested here.
// Every call mirrors a C entry point one to one; errors carry the library's
// text (the reference's Go parse errors for MK_EPARSE).
package mk

// #cgo CFLAGS: -I${SRCDIR}/../../../include
// #cgo LDFLAGS: -L${SRCDIR}/../../../misaka-net_amd/lib -lmisaka_amd -Wl,-rpath,${SRCDIR}/../../../misaka-net_amd/lib
// #include <stdlib.h>
// #include "mk.h"
import "C"

import (
	"fmt"
	"sort"
	"strings"
	"unsafe"
)

// NodeKind is a NODE_INFO type (master.go:431-438) or the master itself.
type NodeKind int

const (
	Program NodeKind = C.MK_NODE_PROGRAM
	Stack   NodeKind = C.MK_NODE_STACK
	Master  NodeKind = C.MK_NODE_MASTER
	// peers of a mixed deployment, served by reference processes (row f4)
	RemoteProgram NodeKind = C.MK_NODE_REMOTE_PROGRAM
	RemoteStack   NodeKind = C.MK_NODE_REMOTE_STACK
)

// Status bits of one /compute result (mk.h MK_ST_*).
const (
	Quiescent     = C.MK_ST_QUIESCENT
	Budget        = C.MK_ST_BUDGET
	StackOverflow = C.MK_ST_STACK_OVERFLOW
	OutputStop    = C.MK_ST_OUTPUT_STOP
	RemoteWait    = C.MK_ST_REMOTE_WAIT
	CallOpen      = C.MK_ST_CALL_OPEN
	HasOutput     = C.MK_ST_HAS_OUTPUT
)

// Node describes one node of a network: its service name, kind and PROGRAM.
type Node struct {
	Name    string
	Kind    NodeKind
	Program string
}

// Options mirrors mk_opts (zero values = library defaults).
type Options struct {
	Budget     uint32
	StackCap   uint32
	Flags      uint32
	DeviceMask uint32
}

func (o Options) c() C.mk_opts {
	return C.mk_opts{budget: C.uint32_t(o.Budget), stack_cap: C.uint32_t(o.StackCap),
		flags: C.uint32_t(o.Flags), device_mask: C.uint32_t(o.DeviceMask)}
}

// Net is a loaded network (mk_net_load); safe for concurrent use.
type Net struct{ h *C.mk_net }

// Load parses and lowers every program node (ProgramNode.LoadProgram,
// program.go:178-193, for each node of NODE_INFO) and resolves names once.
func Load(nodes []Node) (*Net, error) {
	sorted := append([]Node(nil), nodes...)
	sort.Slice(sorted, func(i, j int) bool { return sorted[i].Name < sorted[j].Name })
	descs := make([]C.mk_node_desc, len(sorted))
	var frees []unsafe.Pointer
	defer func() {
		for _, p := range frees {
			C.free(p)
		}
	}()
	cstr := func(s string) *C.char {
		p := C.CString(s)
		frees = append(frees, unsafe.Pointer(p))
		return p
	}
	for i, n := range sorted {
		descs[i] = C.mk_node_desc{name: cstr(n.Name), kind: C.int(n.Kind), program: cstr(n.Program)}
	}
	var h *C.mk_net
	errBuf := make([]byte, 8192)
	rc := C.mk_net_load(&descs[0], C.int(len(descs)), &h, (*C.char)(unsafe.Pointer(&errBuf[0])), C.size_t(len(errBuf)))
	if rc != C.MK_OK {
		return nil, fmt.Errorf("%s", C.GoString((*C.char)(unsafe.Pointer(&errBuf[0]))))
	}
	return &Net{h: h}, nil
}

// Tokenize is tis.Tokenize (tokenizer.go:29-106) on one program: its token
// vectors, or the reference's error text (mk_tokenize).
func Tokenize(program string) ([][]string, error) {
	cs := C.CString(program)
	defer C.free(unsafe.Pointer(cs))
	buf := make([]byte, 64*len(program)+4096)
	rc := C.mk_tokenize(cs, (*C.char)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)))
	text := C.GoString((*C.char)(unsafe.Pointer(&buf[0])))
	if rc == C.MK_EPARSE {
		return nil, fmt.Errorf("%s", text)
	}
	if rc != C.MK_OK {
		return nil, fmt.Errorf("mk_tokenize: %d", int(rc))
	}
	var out [][]string
	for _, line := range strings.Split(text, "\n") {
		out = append(out, strings.Split(line, "\x1f"))
	}
	return out, nil
}

// Close frees the network (after every Sessions of it is closed).
func (n *Net) Close() {
	if n.h != nil {
		C.mk_net_free(n.h)
		n.h = nil
	}
}

// Result of a batch: Out[i] is what /compute would answer for In[i] when
// Status[i]&HasOutput != 0; otherwise the reference's handler would hang.
type Result struct {
	Out    []int32
	Status []uint8
	Steps  []uint32
}

// ComputeBatch evaluates independent /compute inputs (strconv.Atoi values,
// truncated to int32 inside like master.go:237) on the GPU(s).
func (n *Net) ComputeBatch(in []int, opts Options) (*Result, error) {
	r := &Result{Out: make([]int32, len(in)), Status: make([]uint8, len(in)), Steps: make([]uint32, len(in))}
	if len(in) == 0 {
		return r, nil
	}
	in64 := make([]int64, len(in))
	for i, v := range in {
		in64[i] = int64(v)
	}
	o := opts.c()
	rc := C.mk_compute_batch(n.h, (*C.int64_t)(unsafe.Pointer(&in64[0])), C.size_t(len(in)),
		(*C.int32_t)(unsafe.Pointer(&r.Out[0])), (*C.uint8_t)(unsafe.Pointer(&r.Status[0])),
		(*C.uint32_t)(unsafe.Pointer(&r.Steps[0])), &o)
	if rc != C.MK_OK {
		return nil, fmt.Errorf("mk_compute_batch: %d", int(rc))
	}
	return r, nil
}

// Sessions are stateful network instances (row f2): node state, stacks and
// the master's channels persist between Compute calls, as in the reference's
// long-running nodes (program.go:80-92).
type Sessions struct {
	s *C.mk_session
	n int
}

// NewSessions creates n instances on GPU `device` in the post-/reset state.
func (n *Net) NewSessions(device, count int, opts Options) (*Sessions, error) {
	o := opts.c()
	var s *C.mk_session
	if rc := C.mk_session_create(n.h, C.int(device), C.size_t(count), &o, &s); rc != C.MK_OK {
		return nil, fmt.Errorf("mk_session_create: %d", int(rc))
	}
	return &Sessions{s: s, n: count}, nil
}

// Compute performs one /compute call on every instance: in[i] goes to instance i.
func (s *Sessions) Compute(in []int) (*Result, error) {
	if len(in) != s.n {
		return nil, fmt.Errorf("want %d values, got %d", s.n, len(in))
	}
	r := &Result{Out: make([]int32, s.n), Status: make([]uint8, s.n), Steps: make([]uint32, s.n)}
	if s.n == 0 {
		return r, nil
	}
	in64 := make([]int64, s.n)
	for i, v := range in {
		in64[i] = int64(v)
	}
	rc := C.mk_session_compute(s.s, (*C.int64_t)(unsafe.Pointer(&in64[0])), (*C.int32_t)(unsafe.Pointer(&r.Out[0])),
		(*C.uint8_t)(unsafe.Pointer(&r.Status[0])), (*C.uint32_t)(unsafe.Pointer(&r.Steps[0])))
	if rc != C.MK_OK {
		return nil, fmt.Errorf("mk_session_compute: %d", int(rc))
	}
	return r, nil
}

// Cancel abandons every instance's open call (mk_session_cancel): the
// master answered it 504.  What the call set in motion stays.
func (s *Sessions) Cancel() error {
	if rc := C.mk_session_cancel(s.s); rc != C.MK_OK {
		return fmt.Errorf("mk_session_cancel: %d", int(rc))
	}
	return nil
}

// Reset is /reset for every instance (master.go:126-143).
func (s *Sessions) Reset() error {
	if rc := C.mk_session_reset(s.s); rc != C.MK_OK {
		return fmt.Errorf("mk_session_reset: %d", int(rc))
	}
	return nil
}

// Close frees the instances.
func (s *Sessions) Close() {
	if s.s != nil {
		C.mk_session_free(s.s)
		s.s = nil
	}
}

// ComputeSeq performs len(in)/n sequential /compute calls on every instance
// in one launch: in[c*n+i] is call c of instance i (mk_session_compute_seq).
// A master serving concurrent requests on one instance coalesces them here.
func (s *Sessions) ComputeSeq(in []int) (*Result, error) {
	if s.n == 0 || len(in)%s.n != 0 {
		return nil, fmt.Errorf("want a multiple of %d values, got %d", s.n, len(in))
	}
	m := len(in)
	r := &Result{Out: make([]int32, m), Status: make([]uint8, m), Steps: make([]uint32, m)}
	if m == 0 {
		return r, nil
	}
	in64 := make([]int64, m)
	for i, v := range in {
		in64[i] = int64(v)
	}
	rc := C.mk_session_compute_seq(s.s, (*C.int64_t)(unsafe.Pointer(&in64[0])), C.size_t(m/s.n),
		(*C.int32_t)(unsafe.Pointer(&r.Out[0])), (*C.uint8_t)(unsafe.Pointer(&r.Status[0])),
		(*C.uint32_t)(unsafe.Pointer(&r.Steps[0])))
	if rc != C.MK_OK {
		return nil, fmt.Errorf("mk_session_compute_seq: %d", int(rc))
	}
	return r, nil
}

// Step starts a call on instance 0..n-1 (in != nil) or resumes the open
// calls (in == nil): parked on the peers of a mixed deployment, or out of
// their budget slice (status Budget) -- mk_session_step.
func (s *Sessions) Step(in []int) (*Result, error) {
	r := &Result{Out: make([]int32, s.n), Status: make([]uint8, s.n), Steps: make([]uint32, s.n)}
	var p *C.int64_t
	if in != nil {
		if len(in) != s.n {
			return nil, fmt.Errorf("want %d values, got %d", s.n, len(in))
		}
		in64 := make([]int64, s.n)
		for i, v := range in {
			in64[i] = int64(v)
		}
		p = (*C.int64_t)(unsafe.Pointer(&in64[0]))
	}
	rc := C.mk_session_step(s.s, p, (*C.int32_t)(unsafe.Pointer(&r.Out[0])),
		(*C.uint8_t)(unsafe.Pointer(&r.Status[0])), (*C.uint32_t)(unsafe.Pointer(&r.Steps[0])))
	if rc != C.MK_OK {
		return nil, fmt.Errorf("mk_session_step: %d", int(rc))
	}
	return r, nil
}

// RemoteRequest is an outstanding Program.Send / Stack.Push / Stack.Pop of a
// parked call (mk_remote_req).
type RemoteRequest struct {
	Node, Op, Remote, Reg uint32
	Value                 int32
}

// RemoteRequests lists instance inst's outstanding requests (mk_session_remote_poll).
func (s *Sessions) RemoteRequests(inst int) ([]RemoteRequest, error) {
	var reqs [C.MK_MAX_PROGRAM_NODES]C.mk_remote_req
	var cnt C.int
	if rc := C.mk_session_remote_poll(s.s, C.size_t(inst), &reqs[0], C.int(len(reqs)), &cnt); rc != C.MK_OK {
		return nil, fmt.Errorf("mk_session_remote_poll: %d", int(rc))
	}
	out := make([]RemoteRequest, int(cnt))
	for i := range out {
		r := reqs[i]
		out[i] = RemoteRequest{uint32(r.node), uint32(r.op), uint32(r.remote), uint32(r.reg), int32(r.value)}
	}
	return out, nil
}

// RemoteDone reports a request's RPC as completed (the popped value for a pop).
func (s *Sessions) RemoteDone(inst int, node uint32, value int32) error {
	if rc := C.mk_session_remote_done(s.s, C.size_t(inst), C.uint32_t(node), C.int32_t(value)); rc != C.MK_OK {
		return fmt.Errorf("mk_session_remote_done: %d", int(rc))
	}
	return nil
}

// PortPut serves a peer's Program.Send into a local port; busy=true while the
// port is full (program.go:163: the RPC waits).
func (s *Sessions) PortPut(inst int, node, reg uint32, value int32) (busy bool, err error) {
	rc := C.mk_session_port_put(s.s, C.size_t(inst), C.uint32_t(node), C.uint32_t(reg), C.int32_t(value))
	if rc == C.MK_EBUSY {
		return true, nil
	}
	if rc != C.MK_OK {
		return false, fmt.Errorf("mk_session_port_put: %d", int(rc))
	}
	return false, nil
}

// StackPush / StackPop serve a peer's Stack.Push / Stack.Pop on a local
// stack; StackPop reports busy while the stack is empty (stack.go:133-155).
func (s *Sessions) StackPush(inst int, stack uint32, value int32) error {
	if rc := C.mk_session_stack_push(s.s, C.size_t(inst), C.uint32_t(stack), C.int32_t(value)); rc != C.MK_OK {
		return fmt.Errorf("mk_session_stack_push: %d", int(rc))
	}
	return nil
}

func (s *Sessions) StackPop(inst int, stack uint32) (value int32, busy bool, err error) {
	var v C.int32_t
	rc := C.mk_session_stack_pop(s.s, C.size_t(inst), C.uint32_t(stack), &v)
	if rc == C.MK_EBUSY {
		return 0, true, nil
	}
	if rc != C.MK_OK {
		return 0, false, fmt.Errorf("mk_session_stack_pop: %d", int(rc))
	}
	return int32(v), false, nil
}

// NodeIndex is mk_net_node_index: the kind and index of a node by name.
func (n *Net) NodeIndex(name string) (NodeKind, int, error) {
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	var kind, idx C.int
	if rc := C.mk_net_node_index(n.h, cs, &kind, &idx); rc != C.MK_OK {
		return 0, 0, fmt.Errorf("mk_net_node_index %q: %d", name, int(rc))
	}
	return NodeKind(kind), int(idx), nil
}

// TraceEntry is one retired instruction of a traced lane (mk_trace_entry).
type TraceEntry struct {
	Round    uint32
	Node, IP uint16
	Acc, Bak int64
}

// Trace runs one /compute input through the interpreter and returns its
// first max retired instructions (mk_trace_lane) -- the reference's
// per-instruction log.Printf (program.go:222-223) as data.
func (n *Net) Trace(device int, input int, max int, opts Options) ([]TraceEntry, uint8, error) {
	if max <= 0 {
		return nil, 0, fmt.Errorf("max must be positive")
	}
	buf := make([]C.mk_trace_entry, max)
	o := opts.c()
	var cnt C.uint32_t
	var st C.uint8_t
	if rc := C.mk_trace_lane(n.h, C.int(device), C.int64_t(input), &o, &buf[0], C.uint32_t(max), &cnt, &st); rc != C.MK_OK {
		return nil, 0, fmt.Errorf("mk_trace_lane: %d", int(rc))
	}
	out := make([]TraceEntry, int(cnt))
	for i := range out {
		e := buf[i]
		out[i] = TraceEntry{uint32(e.round), uint16(e.node), uint16(e.ip), int64(e.acc), int64(e.bak)}
	}
	return out, uint8(st), nil
}
