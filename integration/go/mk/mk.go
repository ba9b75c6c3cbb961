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
	"unsafe"
)

// NodeKind is a NODE_INFO type (master.go:431-438) or the master itself.
type NodeKind int

const (
	Program NodeKind = C.MK_NODE_PROGRAM
	Stack   NodeKind = C.MK_NODE_STACK
	Master  NodeKind = C.MK_NODE_MASTER
)

// Status bits of one /compute result (mk.h MK_ST_*).
const (
	Quiescent     = C.MK_ST_QUIESCENT
	Budget        = C.MK_ST_BUDGET
	StackOverflow = C.MK_ST_STACK_OVERFLOW
	OutputStop    = C.MK_ST_OUTPUT_STOP
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
