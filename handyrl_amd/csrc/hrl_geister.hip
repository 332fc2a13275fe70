// hrl_geister.hip — batched Geister rules for device self-play (handyrl/envs/geister.py:170-541).
//
// E games advance together in HBM; the state is the one GeisterBatch (envs/geister.py) keeps:
//   board      (E, 36) int8   -1 empty, piece = colour*2 + type (type 0 blue, 1 red), cell = x*6 + y
//   color      (E,)    int64  side to move
//   turn_count (E,)    int64  -2, -1 while the layouts are set, then the move count (200 = draw)
//   win        (E,)    int64  -1 none, 0 black, 1 white, 2 draw
//   cnt        (E, 4)  int64  pieces left per (colour, type)
// As torch ops one ply of rules is ~175 small launches (legal mask ~30, observation ~45, step ~95) at
// E = 2048, each a few microseconds of a mostly idle GPU.  Here each is ONE launch with the same integer
// results (the GPU rules test replays the 24 reference games through these kernels):
//   legal        thread per (game, action label): 214 labels, white's move labels in its 180-degree frame
//   observation  thread per (game, cell): the 7 planes of the viewer, rotated for white, and the 18 scalars
//   step         thread per game: layout placement, move / capture / escape, piece counts, win and draw
// Integer / byte work, HBM-light (a few bytes per game): launch latency is the whole cost.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hrl_env.h"
#include "../../include/hrl_targets.h"

namespace {

constexpr int kCells = 36, kMoves = 144, kLayouts = 70, kActions = kMoves + kLayouts;
constexpr int kMaxMoves = 200;
__device__ __constant__ int kDx[4] = {-1, 0, 0, 1};   // geister.py D = (-1,0), (0,-1), (0,1), (1,0)
__device__ __constant__ int kDy[4] = {0, -1, 1, 0};

// target cell of (direction, cell), -1 off the board
__device__ __forceinline__ int target(int d, int cell) {
    const int nx = cell / 6 + kDx[d], ny = cell % 6 + kDy[d];
    return (nx >= 0 && nx < 6 && ny >= 0 && ny < 6) ? nx * 6 + ny : -1;
}

// off-board step that is a goal of `colour`: black escapes past y = 5, white past y = 0 (x = -1 or 6)
__device__ __forceinline__ bool goal(int colour, int d, int cell) {
    const int nx = cell / 6 + kDx[d], ny = cell % 6 + kDy[d];
    return (nx == -1 || nx == 6) && ny == (colour == 0 ? 5 : 0);
}

__global__ void legal_kernel(const int8_t *__restrict__ board, const int64_t *__restrict__ color,
                             const int64_t *__restrict__ turn_count, int64_t E, uint8_t *__restrict__ legal) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E * kActions) return;
    const int64_t e = i / kActions;
    const int j = (int)(i - e * kActions);
    const bool setting = turn_count[e] < 0;
    bool ok;
    if (j >= kMoves) {
        ok = setting;
    } else if (setting) {
        ok = false;
    } else {
        const int c = (int)color[e];
        const int a = c == 1 ? kMoves - 1 - j : j;   // white's labels are the absolute ones flipped
        const int d = a / kCells, cell = a - d * kCells;
        const int8_t *b = board + e * kCells;
        const int p = b[cell];
        const bool own = p >= 0 && (p >> 1) == c;
        const int t = target(d, cell);
        if (t >= 0) {
            const int q = b[t];
            ok = own && !(q >= 0 && (q >> 1) == c);
        } else {
            ok = own && (p & 1) == 0 && goal(c, d, cell);   // only a blue piece escapes
        }
    }
    legal[i] = ok ? 1 : 0;
}

// Rec: optional episode record of the observation (DeviceGenerator): slot t (read from device memory) of
// planes (E, Tm, 7, 36) / scalar (E, Tm, 18) gets the view when the game is active, zeros otherwise.
struct Rec {
    const uint8_t *active;
    const int64_t *t;
    int64_t Tm;
    float *planes, *scalar;
};

__global__ void observation_kernel(const int8_t *__restrict__ board, const int64_t *__restrict__ color,
                                   const int64_t *__restrict__ cnt, const int64_t *__restrict__ player,
                                   int64_t E, int full, float *__restrict__ planes, float *__restrict__ scalar,
                                   Rec rec) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= E * kCells) return;
    const int64_t e = i / kCells;
    const int cell = (int)(i - e * kCells);
    const int c = (int)color[e];
    const bool turn_view = player[e] == c;
    const int me = turn_view ? c : 1 - c, opp = 1 - me;
    // white sees the board rotated by 180 degrees: its cell k shows absolute cell 35 - k
    const int p = board[e * kCells + (me == 1 ? kCells - 1 - cell : cell)];
    const bool blue_c = p == me * 2, red_c = p == me * 2 + 1;
    const bool own = blue_c || red_c;
    const bool opp_all = p >= 0 && !own;
    const bool blue_o = full && p == opp * 2, red_o = full && p == opp * 2 + 1;
    const float pv[7] = {1.0f, own ? 1.0f : 0.0f, opp_all ? 1.0f : 0.0f, blue_c ? 1.0f : 0.0f,
                         red_c ? 1.0f : 0.0f, blue_o ? 1.0f : 0.0f, red_o ? 1.0f : 0.0f};
    float *o = planes + e * 7 * kCells + cell;
#pragma unroll
    for (int k = 0; k < 7; ++k) o[k * kCells] = pv[k];
    const bool live = rec.planes && rec.active[e];
    const int64_t slot = rec.planes ? e * rec.Tm + *rec.t : 0;
    if (rec.planes) {
        float *r = rec.planes + slot * 7 * kCells + cell;
#pragma unroll
        for (int k = 0; k < 7; ++k) r[k * kCells] = live ? pv[k] : 0.0f;
    }
    if (cell < 18) {   // [me is black, turn view, one-hot counts 1..4 of (my blue, my red, opp blue, opp red)]
        float v;
        if (cell == 0) {
            v = me == 0 ? 1.0f : 0.0f;
        } else if (cell == 1) {
            v = turn_view ? 1.0f : 0.0f;
        } else {
            const int k = cell - 2, which = k >> 2, n = (k & 3) + 1;
            const int side = which < 2 ? me : opp;
            v = cnt[e * 4 + side * 2 + (which & 1)] == n ? 1.0f : 0.0f;
        }
        scalar[e * 18 + cell] = v;
        if (rec.planes) rec.scalar[slot * 18 + cell] = live ? v : 0.0f;
    }
}

__global__ void step_kernel(int8_t *__restrict__ board, int64_t *__restrict__ color, int64_t *__restrict__ turn_count,
                            int64_t *__restrict__ win, int64_t *__restrict__ cnt, const int64_t *__restrict__ action,
                            const uint8_t *active, const int8_t *__restrict__ layout_type,
                            const int64_t *__restrict__ opos, int64_t E, uint8_t *__restrict__ live) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E || !active[e]) return;
    int8_t *b = board + e * kCells;
    int64_t *n = cnt + e * 4;
    const int c = (int)color[e];
    const int64_t a = action[e];
    int64_t w = win[e];
    const int64_t tc = turn_count[e] + 1;
    if (turn_count[e] < 0) {   // set the mover's layout (geister.py:376-381)
        int64_t lay = a - kMoves;
        lay = lay < 0 ? 0 : lay > kLayouts - 1 ? kLayouts - 1 : lay;
        for (int k = 0; k < 8; ++k) b[opos[c * 8 + k]] = (int8_t)(c * 2 + layout_type[lay * 8 + k]);
        n[c * 2] += 4;
        n[c * 2 + 1] += 4;
    } else {                   // move (geister.py:383-394)
        int64_t ab = c == 1 ? kMoves - 1 - a : a;
        ab = ab < 0 ? 0 : ab > kMoves - 1 ? kMoves - 1 : ab;
        const int d = (int)(ab / kCells), src = (int)(ab - d * kCells);
        const int dst = target(d, src);
        const int piece = b[src];
        if (dst < 0) {         // a blue piece leaves by the goal: its owner wins
            n[piece < 0 ? 0 : piece] -= 1;
            w = c;
        } else {
            const int cap = b[dst];
            if (cap >= 0) {    // capture; the last blue taken wins for the capturer, the last red loses
                n[cap] -= 1;
                if (n[cap] == 0) w = (cap & 1) == 0 ? c : 1 - c;
            }
        }
        b[src] = -1;
        if (dst >= 0) b[dst] = (int8_t)piece;
        if (tc >= kMaxMoves && w < 0) w = 2;
    }
    win[e] = w;
    color[e] = 1 - c;
    turn_count[e] = tc;
    if (live) live[e] = w < 0 ? 1 : 0;   // may alias `active`: this thread read active[e] above
}

inline int grid_for(int64_t n) { return (int)((n + 255) / 256); }

}  // namespace

extern "C" {

int hrl_geister_legal(const int8_t *board, const int64_t *color, const int64_t *turn_count, int64_t E,
                      uint8_t *legal, void *stream) {
    if (E == 0) return HRL_OK;
    if (!board || !color || !turn_count || !legal || E < 0) return HRL_EINVAL;
    hipLaunchKernelGGL(legal_kernel, dim3(grid_for(E * kActions)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       board, color, turn_count, E, legal);
    { const hipError_t err = hipGetLastError(); return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err; }
}

int hrl_geister_observation(const int8_t *board, const int64_t *color, const int64_t *cnt, const int64_t *player,
                            int64_t E, int full, float *planes, float *scalar, void *stream) {
    return hrl_geister_observation_record(board, color, cnt, player, E, full, planes, scalar, nullptr, nullptr, 0,
                                          nullptr, nullptr, stream);
}

int hrl_geister_observation_record(const int8_t *board, const int64_t *color, const int64_t *cnt,
                                   const int64_t *player, int64_t E, int full, float *planes, float *scalar,
                                   const uint8_t *active, const int64_t *t, int64_t Tm, float *rec_planes,
                                   float *rec_scalar, void *stream) {
    if (E == 0) return HRL_OK;
    if (!board || !color || !cnt || !player || !planes || !scalar || E < 0) return HRL_EINVAL;
    if (rec_planes && (!rec_scalar || !active || !t || Tm < 1)) return HRL_EINVAL;
    const Rec rec{active, t, Tm, rec_planes, rec_planes ? rec_scalar : nullptr};
    hipLaunchKernelGGL(observation_kernel, dim3(grid_for(E * kCells)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), board, color, cnt, player, E, full, planes, scalar, rec);
    { const hipError_t err = hipGetLastError(); return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err; }
}

int hrl_geister_step(int8_t *board, int64_t *color, int64_t *turn_count, int64_t *win, int64_t *cnt,
                     const int64_t *action, const uint8_t *active, const int8_t *layout_type, const int64_t *opos,
                     int64_t E, uint8_t *live, void *stream) {
    if (E == 0) return HRL_OK;
    if (!board || !color || !turn_count || !win || !cnt || !action || !active || !layout_type || !opos || E < 0)
        return HRL_EINVAL;
    hipLaunchKernelGGL(step_kernel, dim3(grid_for(E)), dim3(256), 0, static_cast<hipStream_t>(stream), board, color,
                       turn_count, win, cnt, action, active, layout_type, opos, E, live);
    { const hipError_t err = hipGetLastError(); return err == hipSuccess ? HRL_OK : HRL_ELAUNCH_BASE - (int)err; }
}

}  // extern "C"
