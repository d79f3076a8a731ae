package gol

// distributor.go for the MI355X engine: a drop-in replacement for the
// reference's gol/distributor.go (AzheeeQAQ/Game-of-life-distributed).  The
// package API (Params, Run, the Event types, util.Cell) and the io goroutine
// with its channel protocol (gol.go, io.go, event.go) are the reference's own
// and stay as they are; this file replaces the turn loop
// (distributor.go:93-173), initializeAliveCells (:212-220), keyPress
// (:223-280), ticker (:283-302), the worker pool (:304-417) and
// calculateAliveCells (:420-432) with calls into libgolhip.so (golhip.go).
// The reference's net/rpc client and server (:44-62, :434-530) are not
// carried over: they abort the run before turn 0 (SURVEY.md §0).
//
// Event stream, as the reference sends it:
//   CellFlipped{0, cell} for every cell alive at load              (:72-80)
//   per turn: CellFlipped{...} for every changed cell, row-major,
//             then TurnComplete                                    (:164, :171)
//   AliveCellsCount every 2 s                                      (:283-302)
//   ImageOutputComplete, FinalTurnComplete, StateChange{Quitting},
//   close(events)                                                  (:193-206)
// The documented contract is the default (DESIGN.md §9): CompletedTurns is
// the number of completed turns (event.go:12-14), CellFlipped.Cell is
// {X: col, Y: row} like FinalTurnComplete, s/q snapshots are taken at a turn
// boundary and not transposed, p sends StateChange{Paused / Executing}, q ends
// the run with StateChange{Quitting} and close(events).  GOL_REF_QUIRKS=1
// reproduces the reference instead: 0-based turns, Cell{X: row, Y: col},
// transposed snapshots, no StateChange on p, os.Exit(0) on q.
//
// Turns run in batches: with its CellFlipped lists (golhip_flip_stream, the
// lists written by the device straight into page-locked memory), 64 turns a
// call; GOLHIP_EVENTS=turns drops the per-cell events (TurnComplete only) and
// =none also the per-turn ones, which lets the engine fuse 256 turns a call.
// Every engine call holds mu, so the ticker, the keys and a pause act between
// batches, at a turn boundary.

import (
	"fmt"
	"os"
	"strconv"
	"sync"
	"time"

	"uk.ac.bris.cs/gameoflife/util"
)

type distributorChannels struct {
	events     chan<- Event
	ioCommand  chan<- ioCommand
	ioIdle     <-chan bool
	ioFilename chan<- string
	ioOutput   chan<- uint8
	ioInput    <-chan uint8
	keyPresses <-chan rune
}

var (
	refQuirks  = os.Getenv("GOL_REF_QUIRKS") == "1"
	cellEvents = os.Getenv("GOLHIP_EVENTS") != "turns" && os.Getenv("GOLHIP_EVENTS") != "none"
	turnEvents = os.Getenv("GOLHIP_EVENTS") != "none"
)

const (
	cellBatch  = 64  // turns per engine call with CellFlipped lists
	fusedBatch = 256 // turns per engine call without them
)

// reported is the turn number an event carries: completed turns, or the
// reference's 0-based turn index in quirks mode (:113, :171, :216).
func reported(completed int) int {
	if refQuirks {
		return completed - 1
	}
	return completed
}

// flipped is the Cell of a CellFlipped event: {X: col, Y: row}, or the
// reference's transposed Cell{j, i} = {X: row, Y: col} in quirks mode (:77, :216).
func flipped(col, row int) util.Cell {
	if refQuirks {
		return util.Cell{X: row, Y: col}
	}
	return util.Cell{X: col, Y: row}
}

// writeImage streams a raster to the io goroutine as out/<name>.pgm (io.go:42-87).
func writeImage(c distributorChannels, name string, raster []byte) {
	c.ioFilename <- name
	c.ioCommand <- ioOutput
	for _, b := range raster {
		c.ioOutput <- b
	}
}

// snapshotRaster is the board for s / q: row-major, or transposed like the
// reference's (*world)[x][y] stream (:234-238, :250-254) in quirks mode.
func snapshotRaster(eng *engine) []byte {
	raster := eng.snapshot()
	if !refQuirks {
		return raster
	}
	t := make([]byte, len(raster))
	for y := 0; y < eng.height; y++ {
		for x := 0; x < eng.width; x++ {
			t[x*eng.height+y] = raster[y*eng.width+x]
		}
	}
	return t
}

func distributor(p Params, c distributorChannels) {
	name := strconv.Itoa(p.ImageWidth) + "x" + strconv.Itoa(p.ImageHeight)
	c.ioFilename <- name
	c.ioCommand <- ioInput
	cells := make([]byte, p.ImageWidth*p.ImageHeight) // row-major, H rows of W bytes
	for i := range cells {
		cells[i] = <-c.ioInput
	}
	eng := newEngine(p, cells)
	defer eng.close()

	for _, cell := range eng.aliveCells() { // :72-80
		c.events <- CellFlipped{CompletedTurns: 0, Cell: flipped(cell.X, cell.Y)}
	}

	var mu sync.Mutex // held by every engine call and by a pause
	turn := 0         // completed turns; written by this goroutine under mu
	finished := make(chan struct{})
	quit := make(chan struct{}) // closed by 'q'
	var helpers sync.WaitGroup

	helpers.Add(1)
	go func() { // ticker (:283-302): the count and its turn come from one engine read
		defer helpers.Done()
		tick := time.NewTicker(2 * time.Second)
		defer tick.Stop()
		for {
			select {
			case <-finished:
				return
			case <-tick.C:
				mu.Lock()
				at, n := eng.aliveCount()
				mu.Unlock()
				c.events <- AliveCellsCount{CompletedTurns: at, CellsCount: n}
			}
		}
	}()

	if c.keyPresses != nil { // keyPress (:223-280); a nil channel never delivers (gol_test.go:34)
		helpers.Add(1)
		go func() {
			defer helpers.Done()
			for {
				var k rune
				select {
				case <-finished:
					return
				case k = <-c.keyPresses:
				}
				switch k {
				case 's', 'q':
					mu.Lock() // a turn boundary: the snapshot is never torn
					t := turn
					fname := name + "x" + strconv.Itoa(t)
					writeImage(c, fname, snapshotRaster(eng))
					mu.Unlock()
					if k == 'q' {
						c.ioCommand <- ioCheckIdle
						<-c.ioIdle
					}
					c.events <- ImageOutputComplete{CompletedTurns: t, Filename: fname}
					if k == 'q' {
						if refQuirks {
							os.Exit(0) // :261
						}
						close(quit)
						return
					}
				case 'p':
					mu.Lock() // the turn loop stops at its next batch boundary
					t := turn
					fmt.Println(t)
					if !refQuirks {
						c.events <- StateChange{CompletedTurns: t, NewState: Paused}
					}
					for resumed := false; !resumed; {
						select {
						case k2 := <-c.keyPresses:
							resumed = k2 == 'p'
						case <-finished:
							resumed = true
						}
					}
					mu.Unlock()
					fmt.Println("Continuing")
					if !refQuirks {
						c.events <- StateChange{CompletedTurns: t, NewState: Executing}
					}
				}
			}
		}()
	}

	stopped := func() bool {
		select {
		case <-quit:
			return true
		default:
			return false
		}
	}
	batch := fusedBatch
	if cellEvents {
		batch = cellBatch
	}
	for turn < p.Turns && !stopped() {
		want := p.Turns - turn
		if want > batch {
			want = batch
		}
		var done int
		var counts []uint64
		var idx []uint32
		mu.Lock()
		if cellEvents {
			done, counts, idx = eng.flipStream(want)
		} else {
			eng.step(want)
			done = want
		}
		first := turn
		turn += done
		mu.Unlock()
		// the batch's events, turn by turn: CellFlipped before TurnComplete (event.go:57)
		off := 0
		for i := 0; i < done; i++ {
			completed := first + i + 1
			if cellEvents {
				for _, v := range idx[off : off+int(counts[i])] {
					c.events <- CellFlipped{CompletedTurns: reported(completed),
						Cell: flipped(int(v)%eng.width, int(v)/eng.width)}
				}
				off += int(counts[i])
			}
			if turnEvents {
				c.events <- TurnComplete{CompletedTurns: reported(completed)}
			}
		}
	}

	close(finished)
	helpers.Wait()
	if stopped() { // 'q' already wrote its snapshot and sent ImageOutputComplete (:244-261)
		c.events <- StateChange{CompletedTurns: turn, NewState: Quitting}
		close(c.events)
		return
	}

	alive := eng.aliveCells() // :180
	fname := name + "x" + strconv.Itoa(p.Turns)
	writeImage(c, fname, eng.snapshot()) // :182-191
	c.events <- ImageOutputComplete{CompletedTurns: p.Turns, Filename: fname}
	c.events <- FinalTurnComplete{CompletedTurns: p.Turns, Alive: alive}
	c.ioCommand <- ioCheckIdle // :200-201
	<-c.ioIdle
	c.events <- StateChange{CompletedTurns: p.Turns, NewState: Quitting}
	close(c.events)
}
