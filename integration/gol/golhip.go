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
// #include <stdio.h>
// #include <stdlib.h>
// #include "golhip.h"
//
// // golhip_last_error() is thread-local and a goroutine may move to another OS
// // thread between two cgo calls, so every checked call returns its status
// // together with the message, read in the same C call (same thread).
// typedef struct { int rc; char msg[320]; } gh_status;
// static gh_status gh_wrap(int rc) {
//     gh_status s;
//     s.rc = rc;
//     s.msg[0] = 0;
//     if (rc != GOLHIP_OK) snprintf(s.msg, sizeof s.msg, "%s", golhip_last_error());
//     return s;
// }
// static gh_status gh_create(int32_t w, int32_t h, golhip_t *out) { return gh_wrap(golhip_create(w, h, 0, 0, out)); }
// static gh_status gh_create_strip(int32_t w, int32_t h, int32_t r0, int32_t rows, int32_t dev, golhip_t *out) {
//     return gh_wrap(golhip_create_strip(w, h, r0, rows, dev, 0, out));
// }
// static gh_status gh_device_count(int32_t *n) { return gh_wrap(golhip_device_count(n)); }
// static gh_status gh_load_bytes(golhip_t h, const uint8_t *c) { return gh_wrap(golhip_load_bytes(h, c)); }
// static gh_status gh_host_alloc(uint64_t b, void **p) { return gh_wrap(golhip_host_alloc(b, p)); }
// static gh_status gh_group_step_ex(golhip_t *hs, int32_t n, int64_t t, int32_t f) {
//     return gh_wrap(golhip_group_step_ex(hs, n, t, f));
// }
// static gh_status gh_step_sync(golhip_t h, int64_t t) {
//     int rc = golhip_step(h, t, 0);
//     return gh_wrap(rc != GOLHIP_OK ? rc : golhip_sync(h));
// }
// static gh_status gh_flip_stream(golhip_t h, int64_t t, void *out, uint64_t cap, uint64_t *counts, int64_t *done,
//                                 uint64_t *n) {
//     return gh_wrap(golhip_flip_stream(h, t, GOLHIP_FLIPS_INDEX, out, cap, counts, done, n));
// }
// static gh_status gh_flips(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n) { return gh_wrap(golhip_flips(h, xy, cap, n)); }
// static gh_status gh_alive_cells(golhip_t h, int32_t *xy, uint64_t cap, uint64_t *n) {
//     return gh_wrap(golhip_alive_cells(h, xy, cap, n));
// }
// static gh_status gh_alive_count(golhip_t h, uint64_t *n, int64_t *t) { return gh_wrap(golhip_alive_count(h, n, t)); }
// static gh_status gh_snapshot_bytes(golhip_t h, uint8_t *out) { return gh_wrap(golhip_snapshot_bytes(h, out)); }
import "C"

import (
	"os"
	"strconv"
	"unsafe"

	"uk.ac.bris.cs/gameoflife/util"
)

// engine is the board of one Run: one libgolhip handle (a whole torus on
// GPU 0) or, with GOL_NGPU=n / GOL_STRIPS=k in the environment (SURVEY 5's
// config row; the README's halo-exchange extension), k row strips on devices
// 0..n-1 (k = n by default) stepped together by golhip_group_step_ex, their
// halo rows moved between the strips' devices by peer copies.  Side channels
// of the strips are gathered in strip order, which is the board's row-major
// order: alive lists and flip lists concatenate, counts add up.
type engine struct {
	hs     []C.golhip_t // one handle per strip, top to bottom
	row0   []int        // first board row of each strip
	width  int
	height int

	flipsP unsafe.Pointer // golhip_host_alloc buffer of cell indices y*width + x
	flips  []uint32       // a Go view of it
	counts []uint64       // per-turn list lengths of the last flipStream
	xy     []int32        // strips: one strip's flip pairs of a turn
}

// check turns a libgolhip status into the reference's fail-fast behaviour
// (util.Check panics, the io goroutine panics on a bad PGM); the message came
// back with the status from the same C call (gh_wrap).
func check(s C.gh_status) {
	if s.rc != C.GOLHIP_OK {
		panic("golhip: " + C.GoString(&s.msg[0]))
	}
}

func envInt(name string, dflt int) int {
	if v, err := strconv.Atoi(os.Getenv(name)); err == nil {
		return v
	}
	return dflt
}

// newEngine replaces the world allocation and fill of distributor.go:66-80:
// cells is the raster the io goroutine sent, row-major, alive <=> 255.
func newEngine(p Params, cells []byte) *engine {
	e := &engine{width: p.ImageWidth, height: p.ImageHeight}
	ngpu := envInt("GOL_NGPU", 1)
	n := envInt("GOL_STRIPS", 0)
	if n <= 0 {
		n = ngpu
	}
	if n > p.ImageHeight {
		n = p.ImageHeight
	}
	if n <= 1 {
		var h C.golhip_t
		check(C.gh_create(C.int32_t(p.ImageWidth), C.int32_t(p.ImageHeight), &h))
		e.hs, e.row0 = []C.golhip_t{h}, []int{0}
	} else {
		var ndev C.int32_t
		check(C.gh_device_count(&ndev))
		devs := ngpu
		if devs > int(ndev) {
			devs = int(ndev)
		}
		if devs < 1 {
			devs = 1
		}
		for i := 0; i < n; i++ {
			r0, r1 := p.ImageHeight*i/n, p.ImageHeight*(i+1)/n
			var h C.golhip_t
			st := C.gh_create_strip(C.int32_t(p.ImageWidth), C.int32_t(p.ImageHeight), C.int32_t(r0),
				C.int32_t(r1-r0), C.int32_t(i%devs), &h)
			if st.rc != C.GOLHIP_OK {
				e.close()
				check(st)
			}
			e.hs = append(e.hs, h)
			e.row0 = append(e.row0, r0)
		}
	}
	for i, h := range e.hs {
		check(C.gh_load_bytes(h, (*C.uint8_t)(unsafe.Pointer(&cells[e.row0[i]*e.width]))))
	}
	return e
}

func (e *engine) close() {
	if e.flipsP != nil {
		C.golhip_host_free(e.flipsP)
		e.flipsP = nil
		e.flips = nil
	}
	for i, h := range e.hs {
		if h != nil {
			C.golhip_destroy(h)
			e.hs[i] = nil
		}
	}
}

// group is the strips' handle array for golhip_group_step_ex (Go memory
// holding C pointers only, valid for the call).
func (e *engine) group(turns int, wantFlips int) {
	check(C.gh_group_step_ex((*C.golhip_t)(unsafe.Pointer(&e.hs[0])), C.int32_t(len(e.hs)), C.int64_t(turns),
		C.int32_t(wantFlips)))
}

// step runs n turns in fused launches (no per-turn side channels).
func (e *engine) step(n int) {
	if len(e.hs) == 1 {
		check(C.gh_step_sync(e.hs[0], C.int64_t(n)))
		return
	}
	e.group(n, 0)
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
	check(C.gh_host_alloc(C.uint64_t(n*4), &p))
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
		first := e.width * e.height // one turn flips at most every cell
		if first > 16<<20 {
			first = 16 << 20
		}
		e.growFlips(first)
	}
	if len(e.counts) < n {
		e.counts = make([]uint64, n)
	}
	if len(e.hs) > 1 {
		return e.stripFlipStream(n)
	}
	var done C.int64_t
	var total C.uint64_t
	call := func() C.gh_status {
		return C.gh_flip_stream(e.hs[0], C.int64_t(n), e.flipsP, C.uint64_t(len(e.flips)),
			(*C.uint64_t)(unsafe.Pointer(&e.counts[0])), &done, &total)
	}
	st := call()
	if st.rc == C.GOLHIP_ERANGE { // the next turn alone needs `total` entries; nothing advanced
		e.growFlips(int(total))
		st = call()
	}
	check(st)
	return int(done), e.counts[:int(done)], e.flips[:int(total)]
}

// stripFlipStream: group turns one at a time (golhip_group_step_ex keeps each
// strip's list of that turn after the step), each strip's list sized first
// (golhip_flips with cap 0) and the buffer grown to fit before it is copied,
// the strips' lists appended in strip order.  Runs all n turns; the buffer
// only ever grows to what the lists need (no worst-case W x H reservation).
func (e *engine) stripFlipStream(n int) (int, []uint64, []uint32) {
	total := 0
	for done := 0; done < n; done++ {
		e.group(1, 1)
		turnN := 0
		for _, h := range e.hs {
			var k C.uint64_t
			if st := C.gh_flips(h, nil, 0, &k); st.rc != C.GOLHIP_OK && st.rc != C.GOLHIP_ERANGE {
				check(st)
			}
			if k == 0 {
				continue
			}
			if len(e.xy) < 2*int(k) {
				e.xy = make([]int32, 2*int(k))
			}
			check(C.gh_flips(h, (*C.int32_t)(unsafe.Pointer(&e.xy[0])), k, &k))
			if need := total + turnN + int(k); need > len(e.flips) {
				e.growFlipsKeep(need, total+turnN)
			}
			for i := 0; i < int(k); i++ {
				e.flips[total+turnN+i] = uint32(int(e.xy[2*i+1])*e.width + int(e.xy[2*i]))
			}
			turnN += int(k)
		}
		e.counts[done] = uint64(turnN)
		total += turnN
	}
	return n, e.counts[:n], e.flips[:total]
}

// growFlipsKeep grows the flip buffer to at least n entries (doubling),
// keeping its first `keep` entries.
func (e *engine) growFlipsKeep(n int, keep int) {
	if n <= len(e.flips) {
		return
	}
	if n < 2*len(e.flips) {
		n = 2 * len(e.flips)
	}
	var p unsafe.Pointer
	check(C.gh_host_alloc(C.uint64_t(n*4), &p))
	nf := (*[1 << 32]uint32)(p)[:n:n]
	copy(nf, e.flips[:keep])
	if e.flipsP != nil {
		C.golhip_host_free(e.flipsP)
	}
	e.flipsP = p
	e.flips = nf
}

// aliveCells is calculateAliveCells (distributor.go:420-432): Cell{X: col, Y: row}, row-major.
func (e *engine) aliveCells() []util.Cell {
	cells := []util.Cell{}
	for _, h := range e.hs {
		var n C.uint64_t
		if st := C.gh_alive_cells(h, nil, 0, &n); st.rc != C.GOLHIP_OK && st.rc != C.GOLHIP_ERANGE {
			check(st)
		}
		if n == 0 {
			continue
		}
		xy := make([]int32, 2*int(n))
		check(C.gh_alive_cells(h, (*C.int32_t)(unsafe.Pointer(&xy[0])), n, &n))
		for i := 0; i < int(n); i++ {
			cells = append(cells, util.Cell{X: int(xy[2*i]), Y: int(xy[2*i+1])})
		}
	}
	return cells
}

// aliveCount is the ticker's len(calculateAliveCells(world)) (:292) with the
// turn it belongs to, read together (the reference reads *turn unlocked, :294);
// strips add their counts (all at the same turn: the caller holds mu).
func (e *engine) aliveCount() (turn int, count int) {
	for _, h := range e.hs {
		var n C.uint64_t
		var t C.int64_t
		check(C.gh_alive_count(h, &n, &t))
		turn, count = int(t), count+int(n)
	}
	return turn, count
}

// snapshot is the board as the 0/255 raster the io goroutine writes (:186-191).
func (e *engine) snapshot() []byte {
	out := make([]byte, e.width*e.height)
	for i, h := range e.hs {
		check(C.gh_snapshot_bytes(h, (*C.uint8_t)(unsafe.Pointer(&out[e.row0[i]*e.width]))))
	}
	return out
}
