/*
 * golrun.h — C-ABI of libgolhost.so, the host-side mirror of the reference's
 * gol.Run (gol/gol.go:12) built on libgolhip.so.
 *
 * golrun_start is `go gol.Run(p, events, keyPresses)` (gol_test.go:34,
 * count_test.go:26): it starts the run on its own thread; golrun_next_event is
 * one receive of `for event := range events` (it returns 0 once the channel is
 * closed and drained); golrun_send_key is `keyPresses <- k`.
 * Event kinds, fields and String() text follow gol/event.go:19-131.
 */
#ifndef GOLRUN_H
#define GOLRUN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* golrun_start flags */
#define GOLRUN_FLAG_KEYS 0x1u            /* create a keyPresses channel (else nil)          */
#define GOLRUN_FLAG_REF_QUIRKS 0x2u      /* reference quirks: 0-based TurnComplete, transposed
                                            CellFlipped and s/q snapshots (DESIGN.md "Quirks") */
#define GOLRUN_FLAG_NO_CELL_EVENTS 0x4u  /* no per-cell CellFlipped (fused turns, fast)     */
#define GOLRUN_FLAG_NO_TURN_EVENTS 0x8u  /* no per-turn TurnComplete                        */

/* event kinds (gol/event.go) */
#define GOLRUN_ALIVE_CELLS_COUNT 0
#define GOLRUN_IMAGE_OUTPUT_COMPLETE 1
#define GOLRUN_STATE_CHANGE 2
#define GOLRUN_CELL_FLIPPED 3
#define GOLRUN_TURN_COMPLETE 4
#define GOLRUN_FINAL_TURN_COMPLETE 5
/* State (event.go:33-38) */
#define GOLRUN_PAUSED 0
#define GOLRUN_EXECUTING 1
#define GOLRUN_QUITTING 2

typedef struct golrun golrun;
typedef golrun *golrun_t;

/* Go's int is 64-bit (event.go:19-68, util/cell.go:4-6): so are these. */
typedef struct golrun_event {
    int32_t kind;
    int32_t new_state;         /* StateChange.NewState                     */
    int64_t completed_turns;   /* GetCompletedTurns()                      */
    int64_t cells_count;       /* AliveCellsCount.CellsCount               */
    int64_t cell_x, cell_y;    /* CellFlipped.Cell                         */
    int64_t alive_len;         /* len(FinalTurnComplete.Alive)             */
    char filename[256];        /* ImageOutputComplete.Filename             */
    char text[288];            /* String()                                 */
} golrun_event_t;

const char *golrun_last_error(void);
/* root: directory with images/<W>x<H>.pgm; output goes to root/out/.
 * events_cap: 0 = unbuffered (as in the tests), 1000 as in main.go:53.
 * ticker_ms: AliveCellsCount period (<= 0: 2000 as distributor.go:285). */
int golrun_start(int64_t turns, int64_t threads, int64_t width, int64_t height, const char *root, int32_t device,
                 uint32_t flags, int32_t events_cap, int32_t ticker_ms, golrun_t *out);
/* 1 = event received, 0 = channel closed and drained, 2 = timeout (timeout_ms >= 0). */
int golrun_next_event(golrun_t r, golrun_event_t *ev, int32_t timeout_ms);
/* Alive list of the last FinalTurnComplete received (alive_len pairs X, Y). */
int golrun_event_cells(golrun_t r, int64_t *xy, uint64_t cap);
/* String() of an event's fields (event.go:72-131); needs no run or device. */
int golrun_event_string(const golrun_event_t *ev, char *out, uint64_t cap);
/* main.go's headless drain loop (main.go:59-66) on the run's own events, for
 * runs whose event streams are too large to hand over one by one: receives
 * until the channel closes and tallies count[kind].  For CellFlipped of
 * completed turn t in 1..turns_cap (documented contract: 1-based turns):
 * flips[t-1] events and digests[t-1] = sum over them, in arrival order, of
 * splitmix64(i) * (Y * width + X + 1), i = 1, 2, ... within the turn
 * (tests/golden/make_fullsize.py ordered_digest).  flips / digests nullable. */
typedef struct golrun_drain_stats {
    uint64_t count[6];     /* events received, by GOLRUN_* kind              */
    int64_t last_turn;     /* CompletedTurns of the last TurnComplete        */
    int64_t final_alive;   /* len(FinalTurnComplete.Alive), 0 if none         */
} golrun_drain_stats_t;
int golrun_drain(golrun_t r, golrun_drain_stats_t *st, uint64_t *flips, uint64_t *digests, int64_t turns_cap,
                 int64_t width);
int golrun_send_key(golrun_t r, uint32_t key);
/* Drains unread events, joins the run; 0 or the panic message in err. */
int golrun_wait(golrun_t r, char *err, uint64_t err_cap);
int golrun_destroy(golrun_t r);

#ifdef __cplusplus
}
#endif
#endif /* GOLRUN_H */
