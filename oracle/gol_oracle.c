/*
 * gol_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Plain-C restatement of the reference's Game of Life hot path
 * (AzheeeQAQ/Game-of-life-distributed, Go).  Nothing in the shipped product
 * (libgolhip.so) links or calls this file; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.
 *
 * Parity pinning: every function below is checked by tests/test_oracle_golden.py
 * against the reference's own fixtures (check/images/<size>x<turns>.pgm, 9 boards, and
 * check/alive/<size>.csv, 3 x 10,000 turns), committed as data under tests/golden/.
 * The reference itself is Go and there is no Go toolchain in this image, so it
 * cannot be compiled into oracle/_ref (see DESIGN.md "Oracle").
 *
 * Board layout: H rows x W columns, row-major bytes, alive <=> byte == 255.
 * The reference stores world[row][col] with len(world) == ImageWidth
 * (gol/distributor.go:66-69), which is only consistent for square boards;
 * all shipped boards are square and this restatement uses the mathematically
 * correct H x W layout.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ALIVE 255u

/* checkNeighbour — gol/distributor.go:382-417.
 * Counts the 8 neighbours equal to 255 with toroidal wrap (the four wrap
 * branches at :398-409 are exactly "index -1 -> last, index n -> 0"). */
static inline int check_neighbour(const uint8_t *w, int W, int H, int row, int col) {
    int n = 0;
    for (int i = row - 1; i <= row + 1; i++) {
        for (int j = col - 1; j <= col + 1; j++) {
            if (i == row && j == col) continue;            /* :390-392 */
            int x = i, y = j;
            if (x < 0) x = H - 1;                          /* :398-403 */
            if (x >= H) x = 0;
            if (y < 0) y = W - 1;                          /* :404-409 */
            if (y >= W) y = 0;
            if (w[(size_t)x * W + y] == ALIVE) n++;        /* :411-413 */
        }
    }
    return n;
}

/* B3/S23 decision — gol/distributor.go:363-375 (serial) and :329-341 (worker):
 * alive (==255) survives with 2 or 3 neighbours, dead becomes alive with 3;
 * output bytes are 0 or 255. */
static inline uint8_t next_cell(uint8_t cell, int n) {
    if (cell == ALIVE) return (n < 2 || n > 3) ? 0 : ALIVE;
    return n == 3 ? ALIVE : 0;
}

/* calculateNextState — gol/distributor.go:350-379 (Threads == 1 path). */
void oracle_step(const uint8_t *in, uint8_t *out, int W, int H) {
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++)
            out[(size_t)r * W + c] = next_cell(in[(size_t)r * W + c], check_neighbour(in, W, H, r, c));
}

/* Run `turns` turns of oracle_step in place (ping-pong internally). */
int oracle_run(uint8_t *board, int W, int H, long turns) {
    size_t n = (size_t)W * H;
    uint8_t *tmp = (uint8_t *)malloc(n);
    if (!tmp) return -1;
    for (long t = 0; t < turns; t++) {
        oracle_step(board, tmp, W, H);
        memcpy(board, tmp, n);
    }
    free(tmp);
    return 0;
}

/* Same as oracle_run but records len(calculateAliveCells(world)) after every
 * turn (what check/alive/<size>.csv tabulates: row k = alive cells after k turns). */
int oracle_run_counts(uint8_t *board, int W, int H, long turns, int64_t *counts) {
    size_t n = (size_t)W * H;
    uint8_t *tmp = (uint8_t *)malloc(n);
    if (!tmp) return -1;
    for (long t = 0; t < turns; t++) {
        oracle_step(board, tmp, W, H);
        memcpy(board, tmp, n);
        int64_t a = 0;
        for (size_t i = 0; i < n; i++) a += board[i] == ALIVE;
        counts[t] = a;
    }
    free(tmp);
    return 0;
}

/* calculateAliveCells — gol/distributor.go:420-432.
 * Row-major list of Cell{X: col, Y: row} for every byte == 255.
 * xy receives (X, Y) pairs; returns the number of cells (xy may be NULL). */
int64_t oracle_alive_cells(const uint8_t *w, int W, int H, int32_t *xy) {
    int64_t k = 0;
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++)
            if (w[(size_t)r * W + c] == ALIVE) {
                if (xy) { xy[2 * k] = c; xy[2 * k + 1] = r; }
                k++;
            }
    return k;
}

/* initializeAliveCells — gol/distributor.go:212-220.
 * Row-major list of every cell whose byte differs between the two boards.
 * The reference emits Cell{j, i} = {X: row, Y: col} (transposed w.r.t.
 * calculateAliveCells); this oracle returns (col, row) pairs and the host
 * layer applies the reference's orientation (see DESIGN.md "Quirks"). */
int64_t oracle_flips(const uint8_t *a, const uint8_t *b, int W, int H, int32_t *xy) {
    int64_t k = 0;
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++)
            if (a[(size_t)r * W + c] != b[(size_t)r * W + c]) {
                if (xy) { xy[2 * k] = c; xy[2 * k + 1] = r; }
                k++;
            }
    return k;
}

/* splitmix64 finaliser: the counter hash used for the synthetic boards of
 * BASELINE configs 2-5 (not in the reference). The device
 * generator (golhip_fill_random) must produce bit-identical boards. */
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* cell (row y, col x) alive <=> (splitmix64(seed ^ (y*W + x)) & 3) == 0 (25%). */
void oracle_fill_random(uint8_t *w, int W, int H, uint64_t seed) {
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            uint64_t idx = (uint64_t)y * (uint64_t)W + (uint64_t)x;
            w[(size_t)y * W + x] = (splitmix64(seed ^ idx) & 3u) == 0 ? ALIVE : 0;
        }
}

/* ---------------------------------------------------------------------------
 * Worker-pool port — the reference's Threads > 1 turn loop, restated with
 * pthreads so it can be timed as the CPU baseline (gol/distributor.go:116-173).
 * Structure kept on purpose (it is what the reference spends its time on):
 *   - a fresh W x H board allocated every turn (:139-142);
 *   - Threads+1 workers (the off-by-one `<=` at :129) started every turn;
 *   - row indices handed out through a shared queue (:124, :134-136);
 *   - workerWorld computes one row into a 1 x W scratch with the branchy
 *     checkNeighbour and returns that row's alive-cell list (:318-347);
 *   - the distributor gathers every row's list and scatters 255s into the new
 *     board (:145-155);
 *   - initializeAliveCells compares old and new boards under the lock (:164).
 * The row channel is an atomic row counter here.  oracle_run_workerpool counts
 * the flip events ("engine only"); gol_port_events.cpp delivers every event
 * through the host mirror's channel, as gol.Run does ("with events").
 * -------------------------------------------------------------------------*/
typedef struct { int32_t x, y; } cell_t;

typedef struct {
    const uint8_t *world;
    int W, H;
    atomic_int next_row;          /* the `images` row-task channel */
    cell_t **row_cells;           /* the `cells` channel, one slot per row */
    int *row_len;
} pool_t;

static void *pool_worker(void *arg) {
    pool_t *p = (pool_t *)arg;
    uint8_t *scratch = (uint8_t *)malloc((size_t)p->W);        /* newWorld[0] :321-322 */
    for (;;) {
        int row = atomic_fetch_add(&p->next_row, 1);
        if (row >= p->H) break;
        int n = 0;
        for (int h = 0; h < p->W; h++) {
            uint8_t nb = next_cell(p->world[(size_t)row * p->W + h],
                                   check_neighbour(p->world, p->W, p->H, row, h));
            scratch[h] = nb;
            n += nb == ALIVE;
        }
        cell_t *list = (cell_t *)malloc(sizeof(cell_t) * (size_t)(n ? n : 1));  /* calculateAliveCells :345 */
        int k = 0;
        for (int h = 0; h < p->W; h++)
            if (scratch[h] == ALIVE) { list[k].x = row; list[k].y = h; k++; }  /* relabel :310-312 */
        p->row_cells[row] = list;
        p->row_len[row] = k;
    }
    free(scratch);
    return NULL;
}

/* One turn of the worker pool (:118-173 without the event sends): returns the
 * freshly allocated next world (:139-142); the caller frees `world`. */
uint8_t *oracle_pool_turn(const uint8_t *world, int W, int H, int threads, pthread_t *tid) {
    size_t n = (size_t)W * H;
    int nworkers = threads + 1;
    pool_t p;
    p.world = world; p.W = W; p.H = H;
    atomic_init(&p.next_row, 0);
    p.row_cells = (cell_t **)calloc((size_t)H, sizeof(cell_t *));
    p.row_len = (int *)calloc((size_t)H, sizeof(int));
    for (int i = 0; i < nworkers; i++) pthread_create(&tid[i], NULL, pool_worker, &p);
    uint8_t *nw = (uint8_t *)calloc(n, 1);                       /* :139-142 */
    for (int i = 0; i < nworkers; i++) pthread_join(tid[i], NULL);
    for (int r = 0; r < H; r++) {                                /* gather + scatter :145-155 */
        for (int k = 0; k < p.row_len[r]; k++)
            nw[(size_t)p.row_cells[r][k].x * W + p.row_cells[r][k].y] = ALIVE;
        free(p.row_cells[r]);
    }
    free(p.row_cells);
    free(p.row_len);
    return nw;
}

/* Runs `turns` turns in place with the worker-pool structure; returns the total
 * number of CellFlipped events the reference would have sent (or -1). */
int64_t oracle_run_workerpool(uint8_t *board, int W, int H, long turns, int threads) {
    size_t n = (size_t)W * H;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)(threads + 1));
    int64_t flips = 0;
    uint8_t *world = (uint8_t *)malloc(n);
    memcpy(world, board, n);
    for (long t = 0; t < turns; t++) {
        uint8_t *nw = oracle_pool_turn(world, W, H, threads, tid);
        for (size_t i = 0; i < n; i++) flips += nw[i] != world[i];   /* initializeAliveCells :212-220 */
        free(world);
        world = nw;
    }
    memcpy(board, world, n);
    free(world);
    free(tid);
    return flips;
}
