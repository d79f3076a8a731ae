package gol

// The cgo binding of libgolhip.so (include/golhip.h), the MI355X engine that
// replaces the reference's turn loop (gol/distributor.go:93-173) and its side
// channels.  Dropped into the reference's gol package together with
// distributor.go from this directory (INTEGRATION.md); this repository is
// expected at ../engine, next to the reference's gol/ directory, with
// libgolhip.so built (make -C engine/game-of-life-distributed_amd/csrc).
//
// Go memory handed to C (the loaded board, the count slices) is only used
// during the call (cgo pointer rules); the flip buffer is C memory
// (golhip_host_alloc: page-locked, written by the device directly).

// #cgo CFLAGS: -I${SRCDIR}/../engine/include
// #cgo LDFLAGS: -L${SRCDIR}/../engine/game-of-life-distributed_amd/golhip -lgolhip -Wl,-rpath,${SRCDIR}/../engine/game-of-life-distributed_amd/golhip
// #include <stdlib.h>
// #include "golhip.h"
import "C"

import (
	"unsafe"

	"uk.ac.bris.cs/gameoflife/util"
)

// engine is one libgolhip handle: the board of one Run on one GPU.
type engine struct {
	h      C.golhip_t
	width  int
	height int

	flipsP unsafe.Pointer // golhip_host_alloc buffer of cell indices y*width + x
	flips  []uint32       // a Go view of it
	counts []uint64       // per-turn list lengths of the last flipStream
}

// check turns a libgolhip status into the reference's fail-fast behaviour
// (util.Check panics, the io goroutine panics on a bad PGM).
func check(rc C.int) {
	if rc != C.GOLHIP_OK {
		panic("golhip: " + C.GoString(C.golhip_last_error()))
	}
}

// newEngine replaces the world allocation and fill of distributor.go:66-80:
// cells is the raster the io goroutine sent, row-major, alive <=> 255.
func newEngine(p Params, cells []byte) *engine {
	var h C.golhip_t
	check(C.golhip_create(C.int32_t(p.ImageWidth), C.int32_t(p.ImageHeight), 0, 0, &h))
	e := &engine{h: h, width: p.ImageWidth, height: p.ImageHeight}
	check(C.golhip_load_bytes(h, (*C.uint8_t)(unsafe.Pointer(&cells[0]))))
	return e
}

func (e *engine) close() {
	if e.flipsP != nil {
		C.golhip_host_free(e.flipsP)
		e.flipsP = nil
		e.flips = nil
	}
	if e.h != nil {
		C.golhip_destroy(e.h)
		e.h = nil
	}
}

// step runs n turns in fused launches (no per-turn side channels).
func (e *engine) step(n int) {
	check(C.golhip_step(e.h, C.int64_t(n), 0))
	check(C.golhip_sync(e.h))
}

func (e *engine) growFlips(n int) {
	if n <= len(e.flips) {
		return
	}
	if e.flipsP != nil {
		C.golhip_host_free(e.flipsP)
		e.flipsP = nil
		e.flips = nil
	}
	var p unsafe.Pointer
	check(C.golhip_host_alloc(C.uint64_t(n*4), &p))
	e.flipsP = p
	e.flips = (*[1 << 32]uint32)(p)[:n:n]
}

// flipStream runs up to n turns, each with its CellFlipped list
// (initializeAliveCells, distributor.go:212-220), and returns how many ran,
// each turn's list length and the lists concatenated in turn order: cell
// indices y*width + x, row-major within a turn.  The batch stops early rather
// than drop an entry; the views are valid until the next call.
func (e *engine) flipStream(n int) (int, []uint64, []uint32) {
	if e.flipsP == nil {
		most := e.width * e.height // one turn flips at most every cell
		if most > 16<<20 {
			most = 16 << 20
		}
		e.growFlips(most)
	}
	if len(e.counts) < n {
		e.counts = make([]uint64, n)
	}
	var done C.int64_t
	var total C.uint64_t
	call := func() C.int {
		return C.golhip_flip_stream(e.h, C.int64_t(n), C.GOLHIP_FLIPS_INDEX, e.flipsP, C.uint64_t(len(e.flips)),
			(*C.uint64_t)(unsafe.Pointer(&e.counts[0])), &done, &total)
	}
	rc := call()
	if rc == C.GOLHIP_ERANGE { // the next turn alone needs `total` entries; nothing advanced
		e.growFlips(int(total))
		rc = call()
	}
	check(rc)
	return int(done), e.counts[:int(done)], e.flips[:int(total)]
}

// aliveCells is calculateAliveCells (distributor.go:420-432): Cell{X: col, Y: row}, row-major.
func (e *engine) aliveCells() []util.Cell {
	var n C.uint64_t
	if rc := C.golhip_alive_cells(e.h, nil, 0, &n); rc != C.GOLHIP_OK && rc != C.GOLHIP_ERANGE {
		check(rc)
	}
	if n == 0 {
		return []util.Cell{}
	}
	xy := make([]int32, 2*int(n))
	check(C.golhip_alive_cells(e.h, (*C.int32_t)(unsafe.Pointer(&xy[0])), n, &n))
	cells := make([]util.Cell, int(n))
	for i := range cells {
		cells[i] = util.Cell{X: int(xy[2*i]), Y: int(xy[2*i+1])}
	}
	return cells
}

// aliveCount is the ticker's len(calculateAliveCells(world)) (:292) with the
// turn it belongs to, read together (the reference reads *turn unlocked, :294).
func (e *engine) aliveCount() (turn int, count int) {
	var n C.uint64_t
	var t C.int64_t
	check(C.golhip_alive_count(e.h, &n, &t))
	return int(t), int(n)
}

// snapshot is the board as the 0/255 raster the io goroutine writes (:186-191).
func (e *engine) snapshot() []byte {
	out := make([]byte, e.width*e.height)
	check(C.golhip_snapshot_bytes(e.h, (*C.uint8_t)(unsafe.Pointer(&out[0]))))
	return out
}
