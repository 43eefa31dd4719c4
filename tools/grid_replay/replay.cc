// Host replay, under AddressSanitizer + UBSan, of the round-1 grid kernel body that faulted at batch 256 (the parent
// of commit 6aff8c2: og_grid_kernel with the generic pointer `int* SI = in_lds ? sitems : CI`), on the keypoint
// arrays of a real batch-256 GPU run (tools/grid_replay/dump.py).  Test infrastructure only.
//
// Each workgroup phase runs as a loop over the 256 thread ids in order (the LDS atomics become plain increments:
// one valid interleaving; every index the kernel forms is order-independent -- a cursor position of cell c always
// lies in [starts[c], starts[c+1])).  The LDS arrays and the global arrays are separate heap blocks of their exact
// sizes, so ASan reports any access past them; every index is also checked against the tighter bound the kernel
// relies on (sort accesses inside their cell's range, scatter positions below nin and frame_cap).
//
// build: g++ -O1 -g -std=c++17 -ffp-contract=off -fsanitize=address,undefined -fno-omit-frame-pointer
//        tools/grid_replay/replay.cc -o /tmp/grid_replay && /tmp/grid_replay gpurun_out/grid_replay.bin
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static const int COLS = 64, ROWS = 48, CELLS = COLS * ROWS, NT = 256, LDS_ITEMS = 8192;
static long long n_checks = 0, n_bad = 0;

#define CHECK(cond, ...)                       \
    do {                                       \
        n_checks++;                            \
        if (!(cond)) {                         \
            if (n_bad++ < 20) {                \
                std::fprintf(stderr, __VA_ARGS__); \
                std::fprintf(stderr, "\n");    \
            }                                  \
        }                                      \
    } while (0)

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp) return 2;
    int B = 0, cap = 0;
    float g[6];
    if (std::fread(&B, 4, 1, fp) != 1 || std::fread(&cap, 4, 1, fp) != 1 || std::fread(g, 4, 6, fp) != 6) return 2;
    const float minX = g[0], minY = g[1], invW = g[4], invH = g[5];
    std::vector<int> counts(B);
    std::vector<float> xy((size_t)B * cap * 2);
    if (std::fread(counts.data(), 4, B, fp) != (size_t)B || std::fread(xy.data(), 4, xy.size(), fp) != xy.size()) return 2;
    std::fclose(fp);
    // global outputs, exact sizes
    int* cell_start = (int*)std::malloc(sizeof(int) * (size_t)B * (CELLS + 1));
    int* cell_items = (int*)std::malloc(sizeof(int) * (size_t)B * cap);
    long long frames_lds = 0, max_nin = 0, max_cell = 0;
    for (int f = 0; f < B; f++) {
        // LDS of the workgroup, exact sizes (separate blocks: ASan redzones between them)
        int* cnt = (int*)std::malloc(sizeof(int) * (CELLS + 1));
        int* wsum = (int*)std::malloc(sizeof(int) * 32);
        int* starts = (int*)std::malloc(sizeof(int) * (CELLS + 1));
        int* sitems = (int*)std::malloc(sizeof(int) * LDS_ITEMS);
        const int n = counts[f];
        CHECK(n >= 0 && n <= cap, "frame %d: count %d outside [0, frame_cap %d]", f, n, cap);
        const float* K = xy.data() + (size_t)f * cap * 2;
        int* CS = cell_start + (size_t)f * (CELLS + 1);
        int* CI = cell_items + (size_t)f * cap;
        for (int tid = 0; tid < NT; tid++)
            for (int c = tid; c < CELLS; c += NT) cnt[c] = 0;
        auto cell = [&](int i, int* out) {
            const int px = (int)std::roundf((K[2 * i] - minX) * invW);
            const int py = (int)std::roundf((K[2 * i + 1] - minY) * invH);
            if (px >= 0 && px < COLS && py >= 0 && py < ROWS) {
                *out = px * ROWS + py;
                return true;
            }
            return false;
        };
        for (int tid = 0; tid < NT; tid++)
            for (int i = tid; i < n; i += NT) {
                int c;
                if (cell(i, &c)) cnt[c] += 1;
            }
        // exclusive scan, 12 cells per thread (og_block_excl_scan over the per-thread sums)
        const int per = CELLS / NT;
        std::vector<int> local((size_t)NT * per), ssum(NT), ex(NT);
        for (int tid = 0; tid < NT; tid++) {
            int s = 0;
            for (int q = 0; q < per; q++) {
                local[tid * per + q] = s;
                s += cnt[tid * per + q];
            }
            ssum[tid] = s;
        }
        int tot = 0;
        for (int tid = 0; tid < NT; tid++) {
            ex[tid] = tot;
            tot += ssum[tid];
        }
        for (int w = 0; w < NT / 64; w++) wsum[w] = 0;  // (the scan's per-wave totals: touched, as in the kernel)
        for (int tid = 0; tid < NT; tid++)
            for (int q = 0; q < per; q++) CS[tid * per + q] = starts[tid * per + q] = ex[tid] + local[tid * per + q];
        CS[CELLS] = starts[CELLS] = tot;
        for (int tid = 0; tid < NT; tid++)
            for (int q = 0; q < per; q++) cnt[tid * per + q] = ex[tid] + local[tid * per + q];  // cursors
        for (int tid = 0; tid < NT; tid++)
            for (int i = tid; i < n; i += NT) {
                int c;
                if (cell(i, &c)) {
                    const int pos = cnt[c]++;
                    CHECK(pos >= starts[c] && pos < starts[c + 1] && pos < tot && pos < cap,
                          "frame %d: scatter position %d of cell %d outside [%d, %d) / nin %d / cap %d", f, pos, c,
                          starts[c], starts[c + 1], tot, cap);
                    CI[pos] = i;
                }
            }
        const int nin = starts[CELLS];
        max_nin = std::max<long long>(max_nin, nin);
        const bool in_lds = nin <= LDS_ITEMS;
        frames_lds += in_lds;
        int* SI = in_lds ? sitems : CI;
        if (in_lds)
            for (int tid = 0; tid < NT; tid++)
                for (int p = tid; p < nin; p += NT) sitems[p] = CI[p];
        for (int tid = 0; tid < NT; tid++)
            for (int c = tid; c < CELLS; c += NT) {
                const int b = starts[c], e = starts[c + 1];
                CHECK(b >= 0 && b <= e && e <= nin, "frame %d: cell %d range [%d, %d) outside [0, %d)", f, c, b, e, nin);
                max_cell = std::max<long long>(max_cell, e - b);
                for (int p = b + 1; p < e; p++) {
                    const int v = SI[p];
                    int q = p - 1;
                    while (q >= b && SI[q] > v) {
                        CHECK(q + 1 >= b && q + 1 < e, "frame %d: sort write %d outside [%d, %d)", f, q + 1, b, e);
                        SI[q + 1] = SI[q];
                        q--;
                    }
                    CHECK(q + 1 >= b && q + 1 < e, "frame %d: sort write %d outside [%d, %d)", f, q + 1, b, e);
                    SI[q + 1] = v;
                }
            }
        if (in_lds)
            for (int tid = 0; tid < NT; tid++)
                for (int p = tid; p < nin; p += NT) CI[p] = sitems[p];
        // the result: a permutation of the in-grid keypoints, ascending inside every cell
        std::vector<char> seen(n > 0 ? n : 1, 0);
        for (int c = 0; c < CELLS; c++)
            for (int p = CS[c]; p < CS[c + 1]; p++) {
                CHECK(CI[p] >= 0 && CI[p] < n, "frame %d: item %d out of range", f, CI[p]);
                if (CI[p] >= 0 && CI[p] < n) {
                    CHECK(!seen[CI[p]], "frame %d: item %d twice", f, CI[p]);
                    seen[CI[p]] = 1;
                }
                if (p > CS[c]) CHECK(CI[p - 1] < CI[p], "frame %d: cell %d not ascending", f, c);
            }
        std::free(cnt);
        std::free(wsum);
        std::free(starts);
        std::free(sitems);
    }
    std::printf("frames %d (frame_cap %d), LDS path %lld, max nin %lld, max keypoints per cell %lld, index checks %lld, "
                "violations %lld\n",
                B, cap, frames_lds, max_nin, max_cell, n_checks, n_bad);
    std::free(cell_start);
    std::free(cell_items);
    return n_bad ? 1 : 0;
}
