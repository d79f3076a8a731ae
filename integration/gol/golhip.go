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
// (util.Check panics, the io goroutine panics on a bad PGM).
func check(rc C.int) {
	if rc != C.GOLHIP_OK {
		panic("golhip: " + C.GoString(C.golhip_last_error()))
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
		check(C.golhip_create(C.int32_t(p.ImageWidth), C.int32_t(p.ImageHeight), 0, 0, &h))
		e.hs, e.row0 = []C.golhip_t{h}, []int{0}
	} else {
		var ndev C.int32_t
		check(C.golhip_device_count(&ndev))
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
			rc := C.golhip_create_strip(C.int32_t(p.ImageWidth), C.int32_t(p.ImageHeight), C.int32_t(r0),
				C.int32_t(r1-r0), C.int32_t(i%devs), 0, &h)
			if rc != C.GOLHIP_OK {
				e.close()
				check(rc)
			}
			e.hs = append(e.hs, h)
			e.row0 = append(e.row0, r0)
		}
	}
	for i, h := range e.hs {
		check(C.golhip_load_bytes(h, (*C.uint8_t)(unsafe.Pointer(&cells[e.row0[i]*e.width]))))
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
	check(C.golhip_group_step_ex((*C.golhip_t)(unsafe.Pointer(&e.hs[0])), C.int32_t(len(e.hs)), C.int64_t(turns),
		C.int32_t(wantFlips)))
}

// step runs n turns in fused launches (no per-turn side channels).
func (e *engine) step(n int) {
	if len(e.hs) == 1 {
		check(C.golhip_step(e.hs[0], C.int64_t(n), 0))
		check(C.golhip_sync(e.hs[0]))
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
	most := e.width * e.height // one turn flips at most every cell
	if e.flipsP == nil {
		first := most
		if first > 16<<20 {
			first = 16 << 20
		}
		if len(e.hs) > 1 {
			first = most // strips: a whole turn's worst case, see below
		}
		e.growFlips(first)
	}
	if len(e.counts) < n {
		e.counts = make([]uint64, n)
	}
	if len(e.hs) > 1 {
		return e.stripFlipStream(n, most)
	}
	var done C.int64_t
	var total C.uint64_t
	call := func() C.int {
		return C.golhip_flip_stream(e.hs[0], C.int64_t(n), C.GOLHIP_FLIPS_INDEX, e.flipsP, C.uint64_t(len(e.flips)),
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

// stripFlipStream: one group turn at a time (golhip_group_step_ex keeps each
// strip's list of that turn), the strips' lists appended in strip order;
// stops before a turn whose worst case would not fit the buffer.
func (e *engine) stripFlipStream(n int, most int) (int, []uint64, []uint32) {
	total, done := 0, 0
	for ; done < n && total+most <= len(e.flips); done++ {
		e.group(1, 1)
		turnN := 0
		for _, h := range e.hs {
			var k C.uint64_t
			if rc := C.golhip_flips(h, nil, 0, &k); rc != C.GOLHIP_OK && rc != C.GOLHIP_ERANGE {
				check(rc)
			}
			if k == 0 {
				continue
			}
			if len(e.xy) < 2*int(k) {
				e.xy = make([]int32, 2*int(k))
			}
			check(C.golhip_flips(h, (*C.int32_t)(unsafe.Pointer(&e.xy[0])), k, &k))
			for i := 0; i < int(k); i++ {
				e.flips[total+turnN+i] = uint32(int(e.xy[2*i+1])*e.width + int(e.xy[2*i]))
			}
			turnN += int(k)
		}
		e.counts[done] = uint64(turnN)
		total += turnN
	}
	return done, e.counts[:done], e.flips[:total]
}

// aliveCells is calculateAliveCells (distributor.go:420-432): Cell{X: col, Y: row}, row-major.
func (e *engine) aliveCells() []util.Cell {
	cells := []util.Cell{}
	for _, h := range e.hs {
		var n C.uint64_t
		if rc := C.golhip_alive_cells(h, nil, 0, &n); rc != C.GOLHIP_OK && rc != C.GOLHIP_ERANGE {
			check(rc)
		}
		if n == 0 {
			continue
		}
		xy := make([]int32, 2*int(n))
		check(C.golhip_alive_cells(h, (*C.int32_t)(unsafe.Pointer(&xy[0])), n, &n))
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
		check(C.golhip_alive_count(h, &n, &t))
		turn, count = int(t), count+int(n)
	}
	return turn, count
}

// snapshot is the board as the 0/255 raster the io goroutine writes (:186-191).
func (e *engine) snapshot() []byte {
	out := make([]byte, e.width*e.height)
	for i, h := range e.hs {
		check(C.golhip_snapshot_bytes(h, (*C.uint8_t)(unsafe.Pointer(&out[e.row0[i]*e.width]))))
	}
	return out
}
