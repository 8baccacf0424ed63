// fsclg.hip -- gfx950 kernels for fscl's CLR sweep scan (search_maxpos batch).
//
// One 768-thread workgroup (12 wave64s; two workgroups per CU, 6 waves per SIMD, 80 KB of LDS
// each) owns one coarse grid cell and runs the whole position bisection of
// scan-chromosome.c:103-139 on chip: the cell's end points (init_scan_result, :58-101), and
// for each point the alpha search of sm-search.c:269-300 as two phases (11 coarse, 14-15
// refine candidates), two bisection levels per alpha search.  A phase evaluates every
// candidate's bidirectional walk (sm-search.c:105-150) as a contiguous index range found by a
// wave-parallel search (log(alpha*d) is monotone in |d|), cuts each walk part into 2048-site
// segments on the aligned 128-site trip grid, deals the segments round-robin to the 12 waves
// (a trip: 128 sites, two per lane, one dwordx4 load of the interleaved site array), and sums
// each walk EXACTLY as the reference's sequential `sm_logl += term` would, in any order:
//
//   inside the binade of the start value N (the window null sum) every sequential add is
//   S += rne(t/u) with u = ulp(N), an integer; ties (t/u = F + 1/2) round to the even running
//   sum, so each tie needs only the PARITY of the prefix, which is a popcount of ballots.
//   Per lane: fp64 sums of R = rint(t/u) and of |R| (exact below 2^51); per segment: a parity
//   bit; per tie: its in-segment prefix parity.  A walk whose partial sums may leave the
//   binade gets a rigorous approximation + error bound, and is re-summed sequentially only if
//   it could be the argmax.
//
// Few-cell launches (the permutation pipeline's blocking batches, the drop-in search_maxalpha)
// give each cell up to 8 workgroups ("split cells") that share the walks' segments and combine
// their sums through per-cell agent-scope exchange areas.  A split cell's
// alpha search also evaluates the refine walks of a guessed coarse winner beside the coarse
// walks, so that a correct guess saves the refine phase (SmemSplit: 64 walk slots; §10.6).
//
// Arithmetic is compiled with contraction off (no FMA fusing): the reference's polynomial and
// log(alpha d) adds are reproduced operation for operation.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include <cmath>
#include <vector>
#include <algorithm>
#include <type_traits>
#include <unordered_map>
#include <chrono>

#include "../../../include/fsclg.h"
#include "cell_order.h"

#pragma clang fp contract(off)

#ifdef FSCLG_TRACE
#define TRACE(...) do { if (blockIdx.x == 0 && threadIdx.x == 0) printf(__VA_ARGS__); } while (0)
#else
#define TRACE(...) do {} while (0)
#endif

namespace {

// 12 waves per workgroup, two workgroups per CU (80 KB LDS each), 6 waves per SIMD: the
// term loop is latency-bound, and occupancy is what hides it (measured: 3 waves/SIMD 25.5
// ms, 4 waves 16.2 ms, 6 waves 15.2 ms per C2 launch)
#ifndef FSCLG_WG
#define FSCLG_WG 768
#endif
#ifndef FSCLG_WPE
#define FSCLG_WPE 6
#endif
#ifndef FSCLG_LDS_WG
#define FSCLG_LDS_WG 81920
#endif
constexpr int WG = FSCLG_WG;
constexpr int NWAVE = WG / 64;
#ifndef FSCLG_SEG
#define FSCLG_SEG 2048
#endif
constexpr int SEG = FSCLG_SEG;     // terms per work segment
#ifndef FSCLG_SEG_SPLIT
#define FSCLG_SEG_SPLIT 1024
#endif
constexpr int SEG_SPLIT = FSCLG_SEG_SPLIT;  // split cells (latency): finer segments spread over the members' waves
constexpr int MAXWALK = 32;        // 2 points x 16 candidates
#ifndef FSCLG_MAXSPLIT
#define FSCLG_MAXSPLIT 8  // members per split cell at most
#endif
constexpr int MAXWALK_SPLIT = 64;  // split cells: 2 points x (11 coarse + 15 speculative refine candidates)
constexpr int MAXSEG_W = (163841 / SEG_SPLIT + 4 + 31) / 32 * 32;  // segments per walk (165 at 163841 terms, split;
                                                                  // each part's ends are 128-site aligned)
constexpr int SEGWORDS = MAXSEG_W / 32;
constexpr int MAXTIES = 512;       // per eval_walks; overflow sends the affected argmax to the exact slow path
constexpr int MAXREF = 16;
constexpr int LDS_WG = FSCLG_LDS_WG;  // LDS per workgroup (default: two workgroups per CU, 160 KiB)

#ifndef FSCLG_U
#define FSCLG_U 2
#endif
#ifndef FSCLG_U_SPLIT
#define FSCLG_U_SPLIT 2
#endif
// terms per lane per loop trip (independent load chains): the throughput kernel's register
// budget allows 2; split cells (latency, few waves per SIMD) may take more per trip
constexpr int U_MAIN = FSCLG_U, U_SPLIT = FSCLG_U_SPLIT;
constexpr int U_MAX = U_MAIN > U_SPLIT ? U_MAIN : U_SPLIT;
constexpr double LOG_AD_MIN = -20.0;  // fscl.h:79
constexpr double LOG_AD_MAX = 4.0;    // fscl.h:80
constexpr int PAD = 1024;             // slack after pos/row: a trip may read up to 2*64*U past a walk's end
static_assert(2 * 64 * U_MAX <= PAD, "look-ahead past the padding");
static_assert(SEG_SPLIT % (64 * U_SPLIT) == 0 && SEG % (64 * U_MAIN) == 0, "segments of whole trips");
constexpr uint32_t POS_BIAS = 0x80000000u;  // positions are stored biased: unsigned order = signed order
static_assert(U_MAIN % 2 == 0 && U_SPLIT % 2 == 0, "the interleaved site array holds two sites per lane per block");

// The site array is interleaved per aligned block of 128 sites (one trip): lane l's 16 bytes
// hold sites l and l + 64 of the block, so a trip's sites are one dwordx4 per lane (one
// vector-memory instruction where two dwordx2 cost two: the texture path takes ~16 cycles per
// wave-instruction whatever its width, HISTORY.md §10.2, vmem_probe).  Site i lives at phys(i).
__host__ __device__ __forceinline__ uint32_t phys(uint32_t i) { return (i & ~127u) | ((i & 63u) << 1) | ((i >> 6) & 1u); }

enum { PF_UNSUPPORTED = 1, PF_NOCONV = 2, PF_SPLIT_TIMEOUT = 4 };
constexpr unsigned int XFAIL_BIT = 0x80000000u;  // split cells: a member's timeout, in the cell's arrival word

struct Params {
  const uint2* pr;             // [n_snps + PAD] (position ^ POS_BIAS, device row = caller's row + 1; 0: zero sentinel)
  const double* logt3;         // [3][65536]: c_b + log_table[i], the three branches of sm-search.c:40-46
  const double* coef;          // [n_iv][2 planes][n_rows + 1][2] (coef_off), device row 0 all zero (sentinel)
  const double* nullrow;       // [n_rows + 1], entry 0 zero
  const double* thr;           // thr[j] = least x with (int)((x - LOG_AD_MIN) / step) >= j, j = 1..n_iv-1
  const int32_t* chr_start;
  const int32_t* chr_n;
  const double* chr_null;      // [n_chr] null sum of a whole chromosome (windows that are the chromosome)
  const double* win_null;      // [n_snps] null sum of the window starting at ws (chromosomes above 2*eval_range+1 SNPs)
  const double* la_coarse;     // [n_coarse]
  const double* la_refine;     // [n_coarse + 1][MAXREF]; row n_coarse: around LOG_AD_MAX
  const int32_t* n_refine;     // [n_coarse + 1]
  const uint32_t* dfail;       // [n_coarse + (n_coarse + 1) * MAXREF]: per alpha, the least |d| with
                               // logt(|d|) + lalpha > LOG_AD_MAX (logt is nondecreasing in |d|)
  const uint32_t* dband;       // [alpha row][n_iv + 1]: the least |d| with logt(|d|) + lalpha >= thr[j] (band cuts)
  int nd;                      // n_iv + 1 (dband's row stride)
  int band_th;                 // a band's window is staged when its pieces hold at least this many trips
  int band_nb;                 // at most this many bands (FSCLG_BAND_NB, experiments; NBMAX by default)
  int band_minp;               // a walk part is cut at a band only where both pieces hold this many trips
  const int32_t* tpos;         // [ceil(n_snps / 128)]: the position of site 128 t (band cut searches)
  int off_bd;                  // band mode: byte offset of its BandLds in the dynamic LDS (after the logt copy;
                               // reserved only when band_th >= 0, so the walk-window path keeps the whole window)
  const fsclg_cell_t* cells;
  fsclg_point_t* out;
  unsigned long long* stats;   // 8 counters
  unsigned long long* ctrace;  // optional per-cell [start, end, cu id, terms, phase ticks x4] (FSCLG_CELL_TRACE)
  unsigned long long* ivhist;  // optional [n_iv]: terms per spline interval, one sample per segment
  int n_coarse;
  int n_iv;
  int n_rows;
  int stride;                  // n_rows + 1
  int pstride;                 // bytes from plane A to plane B of an interval: stride * 16
  double step;
  double inv_step;
  double iv_off;               // -LOG_AD_MIN * inv_step - 1e-9 (interval_of)
  int ivc0;                    // LDS coefficient cache: intervals [ivc0, ivc0 + n_civ), every row
  int n_civ, civ_max;          // civ_max = max(n_civ - 1, 0)
  int n_cache;                 // n_civ * stride blocks
  int off_thr, off_nul;        // byte offsets in fsclg_dyn (the coefficient window at 0)
  int off_lt, lt_hi;           // LDS copy of logt3 branch 2 (|d| > 2^24) entries [256, lt_hi) at off_lt; lt_hi 0: none
  uint32_t lt_span;            // |d| is in that copy iff |d| - 2^24 < lt_span (unsigned); 0: none
  const double* lx;            // FSCLG_LOG_CALC: the mid branch computed (logx_mid), its 256-entry table (LX_BYTES)
  int off_lx, lx_on;           //   at off_lx in LDS; lx_on 0: the mid branch from logt3 (the device check failed)
  int eval_range;
  int bp_resl;
  int n_cells;
  int mode;                    // 0: search_maxpos on cells, 1: search_maxalpha on given points,
                               // 2: search_maxalpha on cell endpoints (epos, two per block) into ept
  const int2* epos;            // mode 2: (chr, position) of each distinct endpoint
  int n_ep;
  fsclg_point_t* ept;          // mode 2 out / mode 0 in: evaluated endpoints
  const int2* cell_ep;         // mode 0: (start, end) endpoint indices of each cell, or null
  // split cells (mode 0): `split` workgroups ("members") per cell share every walk's segments and
  // combine their partial sums through a per-cell exchange area in global memory (XAcc, two
  // regions used in turn) and a per-cell arrival counter (zeroed before the launch)
  int lookahead;               // mode 0: evaluate the next bisection level's predicted midpoint
                               // beside the current one (FSCLG_LOOKAHEAD=0: one point per search;
                               // 2: mispredict on purpose, the fallback path's test)
  int split;                   // members per cell (1: one workgroup per cell)
  int spec_refine;             // split cells: evaluate the refine walks of a guessed coarse winner beside the
                               // coarse walks (one phase per alpha search when the guess holds)
  int ci_guess;                // the guess for points with no evaluated neighbour (the recent results' mode)
  char* xacc;                  // [n_cells][2] XAcc
  unsigned int* xcnt;          // [n_cells] arrivals; bit 31: some member of the cell timed out (XFAIL_BIT)
  unsigned long long xwait;    // split cells: wall-clock ticks (100 MHz) a member waits for the others
  unsigned long long xdelay;   // tests only (FSCLG_TEST_SPLIT_DELAY_US): member 0 of cell 0 sleeps this
                               // long before its first arrival, so that the other members time out
};

struct Pt {                     // one scan point being evaluated (scan_pt_t subset)
  int chr, nearest, sweep, wstart, wend, n_snps, flags, pad;
  int ci;                        // its alpha search's coarse winner (n_coarse: none beat the initial state)
  int sg;                        // split cells: the coarse winner guessed before the search (speculative refine)
  int spad;                      // split cells: (first << 8) | count of the speculative refine walks
  int pad2;
  double N, inv_u, u, la, sm, clr;
};

struct Walk {
  int p;          // point slot
  int nl, nr;     // terms left / right of the nearest SNP
  int len;        // 0 (nearest already outside log(ad) <= 4) or 1 + nl + nr
  int seg0;       // first global segment id
  int nseg;       // left-part segments then right-part segments (seg_bounds)
  int nsl;        // left-part segments
  int wb;         // LDS coefficient window base for this walk
  double la;
  double xl, xr;  // log(alpha d) at the walk's far ends (the walk's largest x is one of them)
  uint32_t dfail; // a site is outside the walk iff its |d| >= dfail (Params::dfail)
  int kd;         // the walk's alpha row in Params::dfail / Params::dband
};

// band mode (the throughput kernel): a phase's walks are evaluated interval band by
// band.  Band b holds the intervals [bbase[b], bbase[b] + K) (K: the LDS window), the bands tile
// downwards from the top interval of the phase's walks, and below the last one lies the remainder.
// A walk part's sites in band b are those with |d| in [D(bbase[b]), D(bbase[b - 1])) (Params::dband):
// one contiguous run of sites, a "piece", found as a trip range (cut[]: the trip holding the cut,
// relative to the part's first trip; -1: the part never reaches the band) whose boundary trips
// are masked by the same |d| test ("lazy cuts", run_piece_seg).  Pieces are cut into segments of
// TPS trips; sb[] numbers a walk's segments in site-index order (left part's pieces from band 0 down
// to the remainder, then the right part's from the remainder up to band 0).
#ifndef FSCLG_NBMAX
#define FSCLG_NBMAX 8
#endif
constexpr int NBMAX = FSCLG_NBMAX;
constexpr int NPIECE = 2 * (NBMAX + 1);  // pieces per walk
struct BandLds {
  alignas(16) int16_t cut[MAXWALK][2][NBMAX];  // -1: the part never reaches the band; -2: dropped (pieces merged)
  uint32_t dv[MAXWALK][NBMAX];      // the walk's |d| bound of each band (Params::dband)
  int8_t qof[MAXWALK][2][NBMAX + 1];  // the piece of (walk, part) that group g processes, -1: none
  uint8_t sb[MAXWALK][NPIECE + 1];
  int bbase[NBMAX];
  int nb;
  int nrun;
  int run_g0[NBMAX + 2];            // run r: groups (= bands, nb: the remainder) [run_g0[r], run_g0[r + 1])
  int run_stage[NBMAX + 1];         // run r stages band run_g0[r]'s window first (0: keeps the loaded one)
  int gitems[NBMAX + 1];            // segments per group
  int gtrips[NBMAX + 1];            // trips per group
};

template <int MW, bool BAND = false>
struct SmemT {
  static constexpr int MAXW = MW;
  static constexpr bool HAS_BAND = BAND;
  Pt pt[4];                       // cells: start, end, midpoint, the midpoint's predicted child
  Walk w[MW];
  unsigned long long P[MW];
  unsigned long long Q[MW];
  double Pd[MW], Qd[MW];  // fp64 sums of the lanes whose accumulators passed 2^51 (approximate)
  unsigned int segbits[MW][SEGWORDS];
  int wflag[MW];
  int exact[MW];
  double val[MW];
  double appr[MW];
  double bnd[MW];
  int ties[MAXTIES];
  int n_ties;
  int seg_total;
  int nwalk;
  int need_slow[MW];
  int n_slow;
  int best[3];
  unsigned long long cnt[8];
  int ivc0;                       // base interval of the coefficient window now in LDS
  int ngrp;                       // walk groups of the phase (one LDS window each), in segment order
  int gwb[MW];
  int gseg[MW + 1];
  int gk[MW + 1];                 // the group's walks: word[gk[g] .. gk[g + 1])
  int word[MW];              // walks in segment order
  int hkey;                       // interval-histogram key of the phase: 0 coarse, 1 + c refine around coarse c
  int hitmask;                    // split cells: the points whose speculative refine walks were the right ones
  unsigned long long tph[5];      // FSCLG_PHASE_TIMING: wall-clock ticks in bounds / layout / segments / resolve,
                                  // and (slot 4) the split combine's wait for the other members' arrival
  int cell, member;               // split cells: this workgroup's cell and member index
  int inst;                       // split cells: eval_walks instances so far (the XAcc region in turn)
  int xbase;                      // split cells: this member's first tie slot
  int xfail;                      // split cells: PF_SPLIT_TIMEOUT if a member never arrived
  int iev;                        // FSCLG_INST_TRACE: events recorded so far
  int xnt[FSCLG_MAXSPLIT];        // split cells: each member's tie count of the instance
};
using Smem = SmemT<MAXWALK>;             // the throughput kernel (its LDS window takes the rest)
using SmemBand = SmemT<MAXWALK, true>;   // the same in band mode: a kernel of its own, so that band mode's
                                         // layout code does not raise the walk-window kernel's registers
static_assert(sizeof(Smem) == sizeof(SmemBand), "band mode's LDS block is dynamic (Params::off_bd)");
using SmemSplit = SmemT<MAXWALK_SPLIT>;  // split cells: room for speculative refine walks (no LDS window)


// FSCLG_INST_TRACE (development aid): thread 0 of cell 0's first member records timestamped
// events (tag, a, b) after the per-cell trace area: [count, then 4 words per event]
#ifdef FSCLG_INST_TRACE
#define IEV(tag, a, b) do { \
    if (P.ctrace && S.cell == 0 && S.member == 0 && threadIdx.x == 0 && S.iev < 4000) { \
      unsigned long long* q_ = P.ctrace + 8 * (size_t)P.n_cells; \
      const int k_ = S.iev++; \
      q_[1 + 4 * k_] = wall_clock64(); q_[2 + 4 * k_] = (tag); q_[3 + 4 * k_] = (unsigned long long)(a); \
      q_[4 + 4 * k_] = (unsigned long long)(b); q_[0] = (unsigned long long)S.iev; \
    } } while (0)
#else
#define IEV(tag, a, b) do { } while (0)
#endif

// a split cell's exchange area for one instance: every member writes its own slots with plain
// stores (no zeroing, no read-modify-write); after the arrival counter every member reads all
// members' slots and combines them the same way -- integer sums in any order (exact), the
// segments' parity bits by XOR (each segment has one member), the fp64 sums of lanes past 2^51
// in member order, the ties concatenated.  Two areas used in turn: a member writes instance
// i + 2 only after every member has arrived at i + 1, i.e. has finished reading i.
constexpr int MAXSPLIT = FSCLG_MAXSPLIT;
constexpr int XTIES = MAXTIES / MAXSPLIT;  // tie slots per member (more: the overflow path)
struct XAcc {
  unsigned long long P[MAXSPLIT][MAXWALK_SPLIT], Q[MAXSPLIT][MAXWALK_SPLIT];
  double Pd[MAXSPLIT][MAXWALK_SPLIT], Qd[MAXSPLIT][MAXWALK_SPLIT];
  unsigned int wflag[MAXSPLIT][MAXWALK_SPLIT];
  unsigned int segbits[MAXSPLIT][MAXWALK_SPLIT][SEGWORDS];
  unsigned int nt[MAXSPLIT];
  int ties[MAXSPLIT][XTIES];
};

// dynamic LDS of a workgroup (LDS = true): coefficient planes of the top K intervals, the
// interval thresholds and the null rows (offsets in Params)
extern __shared__ __attribute__((aligned(16))) char fsclg_dyn[];

// a trip's two sites of this lane: block bs (a multiple of 128), sites bs + lane, bs + 64 + lane
__device__ __forceinline__ uint4 ld_trip(const uint2* base, uint32_t bs, int lane) {
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(base) + ((bs + 2u * (uint32_t)lane) << 3));
}

__device__ __forceinline__ int pos_at(const Params& P, int i) { return (int)(P.pr[phys(i)].x ^ POS_BIAS); }

// log of |d| as sm-search.c:40-46: three branches, each c_b + log_table[|d| >> 8b], merged
// into one precomputed table (the host forms c_b + log_table[i] with the same IEEE add)
__device__ __forceinline__ double logt_dev(uint32_t ad, const double* __restrict__ LT3) {
  const uint32_t sh = ad > 0xFFFFFFu ? 16u : (ad > 0xFFFFu ? 8u : 0u);
  const uint32_t ix = (ad >> sh) + (sh << 13);  // + 65536 * branch
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(LT3) + (ix << 3));
}

// logt_dev with the far branch (|d| > 2^24: log_table[|d| >> 16] + c_2, where most terms of
// the long walks fall) read from the workgroup's LDS copy; lanes outside it (and the rare
// entries past lt_hi) take the global table
template <bool LDS>
__device__ __forceinline__ double logt_lds(uint32_t ad, const Params& P) {
  if constexpr (LDS) {
    const uint32_t i2 = ad >> 16;
    if (ad > 0xFFFFFFu && i2 < (uint32_t)P.lt_hi)
      return reinterpret_cast<const double*>(fsclg_dyn + P.off_lt)[i2];  // off_lt is pre-offset by -256 entries
  }
  return logt_dev(ad, P.logt3);
}

// FSCLG_LOG_CALC: the mid branch of logt (sm-search.c:43: 5.545177444479562 + log_table[|d| >> 8],
// i = |d| >> 8 in [256, 65536)) computed instead of gathered from the 512 KB table.  i = 2^e m,
// m = i << (15 - e) in [2^15, 2^16); c = the top 9 bits of m (256 choices, k), r = (m - c) / c
// with |r| < 2^-8: log(i) = log(c) - (15 - e) ln2 + log1p(r), log(c) tabulated as hi + lo,
// (15 - e) ln2_hi exact (42-bit ln2_hi), log1p(r) = r - r^2/2 + r^3 (1/3 - r/4 + r^2/5 - r^3/6).
// The host evaluates the same operations for all 65 280 i against the reference's table
// (logx_table: glibc's log, the same IEEE add), adjusts the lo parts of the few k whose entries
// round the other way, and the device checks every entry once (logx_check_kernel): every
// value is the table's, bit for bit, or the path stays off.
constexpr int LX_BYTES = 256 * 32;  // per k: log(c) hi, lo, RN(1/c), pad
#ifndef FSCLG_LOG_CALC
#define FSCLG_LOG_CALC 0
#endif
// FSCLG_LOG_CALC=1: in the split kernel only (the latency-bound tail); 2: in every kernel
template <class SM> constexpr bool lx_kernel() {
  return FSCLG_LOG_CALC >= 2 || (FSCLG_LOG_CALC == 1 && std::is_same<SM, SmemSplit>::value);
}
constexpr double LX_LN2_HI = 0x1.62e42fefa38p-1, LX_LN2_LO = 0x1.ef35793c7673p-45;
__host__ __device__ __forceinline__ double logx_mid(uint32_t i, const double* lx) {
  const int e = 31 - __builtin_clz(i);
  const int n = 15 - e;
  const uint32_t m = i << n;
  const uint32_t k = (m >> 7) & 255u;
  const double lch = lx[4 * k], lcl = lx[4 * k + 1], inv = lx[4 * k + 2];
  const double f = (double)(m & 127u), dn = (double)n;
  const double rh = f * inv;
  const double A = __builtin_fma(-dn, LX_LN2_HI, lch);  // exact
  const double q = __builtin_fma(-dn, LX_LN2_LO, lcl);
  const double sh = A + rh;
  const double t = (A - sh) + rh;
  const double r2 = rh * rh;
  double p = __builtin_fma(rh, -1.0 / 6, 1.0 / 5);
  p = __builtin_fma(rh, p, -1.0 / 4);
  p = __builtin_fma(rh, p, 1.0 / 3);
  const double r3 = r2 * rh;
  p = r3 * p;
  double lo = t + q;
  lo = __builtin_fma(-0.5, r2, lo);
  lo = lo + p;
  const double L = sh + lo;
  return 5.545177444479562 + L;
}

// every mid-branch entry computed on the device against the uploaded table: mismatches counted
__global__ void __launch_bounds__(256) logx_check_kernel(const double* __restrict__ lx, const double* __restrict__ lt3,
                                                         unsigned long long* __restrict__ bad) {
  const uint32_t i = 256u + blockIdx.x * 256u + threadIdx.x;
  if (i < 0x10000u && logx_mid(i, lx) != lt3[0x10000u + i]) atomicAdd(bad, 1ull);
}

// |pos_i - sweep| from biased positions: one v_sad_u32
__device__ __forceinline__ uint32_t absdist(uint32_t upos, uint32_t usweep) {
  uint32_t d;
  asm("v_sad_u32 %0, %1, %2, 0" : "=v"(d) : "v"(upos), "v"(usweep));
  return d;
}

__device__ __forceinline__ double log_ad_of(int i, int sweep, double la, const Params& P) {
  return logt_dev(absdist(P.pr[phys(i)].x, (uint32_t)sweep ^ POS_BIAS), P.logt3) + la;
}

// spline interval of sm-spline.c:52-54, (int)((x - LOG_AD_MIN) / step) clamped, without the
// division: an fma estimate lowered by 1e-9 (its error and the reference's rounding are
// ~1e-13) is the interval or the one below it, and the exact threshold of the next one
// settles it (thr[n_iv] = +inf: the reference clamps at n_iv - 1)
template <bool LDS, class SM>
__device__ __forceinline__ int interval_of(double x, const SM& S, const Params& P) {
  // x >= LOG_AD_MIN (log_table >= 0 and every alpha >= LOG_AD_MIN, checked by
  // fsclg_set_alpha_grid), so the estimate is >= -1e-9 and truncates to >= 0
  int iv = (int)__builtin_fma(x, P.inv_step, P.iv_off);
  iv = min(iv, P.n_iv - 1);
  double hi;
  if constexpr (LDS) hi = reinterpret_cast<const double*>(fsclg_dyn + P.off_thr)[iv + 1];
  else hi = P.thr[iv + 1];
  return iv + (x >= hi ? 1 : 0);
}

template <bool LDS, class SM>
__device__ __forceinline__ double null_of(uint32_t r, const SM& S, const Params& P) {
  if constexpr (LDS) return reinterpret_cast<const double*>(fsclg_dyn + P.off_nul)[r];
  else return P.nullrow[r];
}

// coefficient block of (row, interval).  Layout [iv][plane][row][2]: per interval, plane A
// holds (c0, c1) of every row and plane B (c2, c3), 16 B per entry, so in a ds_read_b128 the
// rows of a 16-lane group fall on 16 distinct 4-bank slots (a 32-B block per row gave 8),
// halving the expected bank conflicts of the random-row gathers; interval-major, so the lanes
// of a wave (neighbouring sites, nearly equal log distance) read from one interval.  The
// byte offset of (iv, r) in plane A is (iv * stride) * 32 + r * 16, plane B adds
// P.pstride = stride * 16; 32-bit offsets (the table is < 4 GiB, checked on upload).
__device__ __forceinline__ uint32_t coef_off(uint32_t r, int iv, const Params& P) {
  return (__umul24((uint32_t)iv, (uint32_t)P.stride) << 5) + (r << 4);
}

__device__ __forceinline__ void coef_ld(const char* base, uint32_t off, const Params& P, double2& a, double2& b) {
  a = *reinterpret_cast<const double2*>(base + off);
  b = *reinterpret_cast<const double2*>(base + off + (uint32_t)P.pstride);
}


// the coefficient block of (row, interval) into a = (c0, c1), b = (c2, c3): from the LDS
// window when (interval, row) lies in it (every row of intervals [ivc0, ivc0 + n_civ)),
// from the global table otherwise
template <bool LDS, class SM>
__device__ __forceinline__ void coef_fetch(uint32_t r, int iv, const SM& S, const Params& P, double2& a, double2& b) {
  if constexpr (LDS) {
    const uint32_t ci = (uint32_t)(iv - S.ivc0);
    const bool hit = ci < (uint32_t)P.n_civ;  // every row is cached
    coef_ld(fsclg_dyn, coef_off(r, (int)min(ci, (uint32_t)P.civ_max), P), P, a, b);
    if (!hit) coef_ld(reinterpret_cast<const char*>(P.coef), coef_off(r, iv, P), P, a, b);
  } else {
    coef_ld(reinterpret_cast<const char*>(P.coef), coef_off(r, iv, P), P, a, b);
  }
}

// coefficients of U terms: the intervals of all U first (their threshold reads overlap),
// then per term the LDS window or, for lanes outside it, the global table
template <bool LDS, int U, class SM>
__device__ __forceinline__ void coef_stage(const double (&x)[U], const uint32_t (&rv)[U], const SM& S,
                                           const Params& P, int ivc0, double2 (&ca)[U], double2 (&cb)[U],
                                           int (&iv)[U]) {
  constexpr bool CACHE = LDS;
#pragma unroll
  for (int u = 0; u < U; u++) iv[u] = interval_of<LDS>(x[u], S, P);
  if constexpr (CACHE) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t ci = (uint32_t)(iv[u] - ivc0);
#ifdef FSCLG_EXP_COEF_LDS  // timing ablation (wrong results): every coefficient from the LDS window
      if (P.n_civ > 0)
        coef_ld(fsclg_dyn, coef_off(rv[u], (int)min(ci, (uint32_t)P.civ_max), P), P, ca[u], cb[u]);
#else
      if (ci < (uint32_t)P.n_civ)  // every row is cached
        coef_ld(fsclg_dyn, coef_off(rv[u], (int)ci, P), P, ca[u], cb[u]);
#endif
      else
        coef_ld(reinterpret_cast<const char*>(P.coef), coef_off(rv[u], iv[u], P), P, ca[u], cb[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; u++)
      coef_ld(reinterpret_cast<const char*>(P.coef), coef_off(rv[u], iv[u], P), P, ca[u], cb[u]);
  }
}

// snp_likelihood (sm-search.c:85-103) with spline_interpolate (sm-spline.c:48-60)
template <bool LDS, class SM>
__device__ __forceinline__ double term_dev(int i, int sweep, double la, const SM& S, const Params& P) {
  const double x = log_ad_of(i, sweep, la, P);
  const int iv = interval_of<LDS>(x, S, P);
  const uint32_t r = P.pr[phys(i)].y;
  double2 a, b;
  coef_fetch<LDS>(r, iv, S, P, a, b);
  const double y = x * (a.x * x * x + a.y * x + b.x) + b.y;
  return y - null_of<LDS>(r, S, P);
}

__device__ __forceinline__ int walk_index(int k, int nearest, int nl) {
  return k == 0 ? nearest : (k <= nl ? nearest - k : nearest + (k - nl));
}

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Narrow the open range (lo, hi) of a predicate T that holds on a prefix of it (lo counts as
// true, hi as false) to hi = lo + 1 with an aligned group of G lanes of one wave: each round
// probes G indices spread over (lo, hi), so ceil(log_{G+1}(hi - lo)) dependent rounds instead
// of log2.  Every lane of the wave calls it (groups with nothing to search pass hi = lo + 1).
// Returns hi, the first index where T is false.
template <int G, typename F>
__device__ __forceinline__ int group_search(int lo, int hi, int lane, F pred) {
  const int j = lane & (G - 1), sh = lane & (64 - G);
  for (;;) {
    const bool act = hi - lo > 1;
    if (!__any(act)) break;
    const long long span = (long long)(hi - lo - 1);
    bool t = false;
    if (act) t = pred(lo + 1 + (int)((span * j) / G));
    const unsigned long long b = __ballot(t);
    if (act) {
      const unsigned long long gm = G == 64 ? b : ((b >> sh) & ((1ull << (G & 63)) - 1));
      const int c = __popcll(gm);  // the probes are nondecreasing: T holds on the first c
      const int nlo = c > 0 ? lo + 1 + (int)((span * (c - 1)) / G) : lo;
      const int nhi = c < G ? lo + 1 + (int)((span * c) / G) : hi;
      lo = nlo; hi = nhi;
    }
  }
  return hi;
}

// init_scan_result (scan-chromosome.c:58-101) for one point by one wave: search_snppos
// (scan-chromosome.c:39-56) ends with j = the least index in [1, n) whose position is >= pos
// (n if none) and i = j - 1; a 64-way search finds the same j
__device__ __forceinline__ void init_point_wave(Pt& pt, int chr, int pos, const Params& P, int lane) {
  const int a = P.chr_start[chr], n = P.chr_n[chr];
  const int j = group_search<64>(0, n, lane, [&](int m) { return pos_at(P, a + m) < pos; });
  if (lane != 0) return;
  const int i = j - 1;
  int near;
  if (j == n) near = n - 1;
  else if ((long long)pos - pos_at(P, a + i) < (long long)pos_at(P, a + j) - pos) near = i;
  else near = j;
  near += a;
  // Q3: the de-collision loop compares a global index with the chromosome's count
  for (int ii = near; ii < n && pos_at(P, ii) == pos; ii++) pos++;
  const int cs = a, ce = a + n - 1, er = P.eval_range;
  int ws, we;
  if (near - er < cs) {
    ws = cs; we = cs + er * 2; if (we > ce) we = ce;
  } else if (near + er > ce) {
    we = ce; ws = ce - er * 2; if (ws < cs) ws = cs;
  } else {
    ws = near - er; we = near + er;
  }
  pt.chr = chr; pt.nearest = near; pt.sweep = pos; pt.wstart = ws; pt.wend = we;
  pt.n_snps = we - ws + 1;
  pt.flags = 0;
  pt.N = (ws == cs && we == ce) ? P.chr_null[chr] : P.win_null[ws];
}

// binade constants of the start value N: |N| in [2^e, 2^(e+1)), u = 2^(e-52)
__device__ __forceinline__ void set_binade(Pt& pt) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(pt.N);
  const int be = (int)((bits >> 52) & 0x7FF);
  const int e = be - 1023;
  if (be == 0 || be == 0x7FF || pt.N >= 0.0) {  // zero / subnormal / inf / non-negative: no integer path
    pt.u = 0.0; pt.inv_u = 0.0;
    return;
  }
  pt.u = __longlong_as_double((long long)(be - 52 > 0 ? be - 52 : 1) << 52);
  pt.inv_u = __longlong_as_double((long long)(1023 + 52 - e) << 52);
}

// walk_bounds for every walk side of the phase: G lanes per (walk, side), a (G+1)-way search
// of the same monotone predicates as sm-search.c:112-147's loops (left: the site is outside,
// log(alpha d) > 4, on a prefix of (wstart - 1, near); right, when the first right neighbour
// is inside: inside on a prefix of (near + 1, wend + 1)).  logt is nondecreasing in |d|, so
// log(alpha d) > 4 is |d| >= dfail, an integer compare per probe (no log-table gather in the
// search's dependent rounds; the host derives dfail from the same table and adds).
template <int G, class SM>
__device__ __forceinline__ void walk_bounds_g(SM& S, const Params& P, int tid, int nw) {
  const int lane = tid & 63, g = tid / G;
  const bool act = g < 2 * nw;
  const int w = act ? g >> 1 : 0, side = g & 1;
  const Walk& W = S.w[w];
  const Pt& pt = S.pt[act ? W.p : 0];
  const int near = pt.nearest;
  const uint32_t usweep = (uint32_t)pt.sweep ^ POS_BIAS, df = W.dfail;
  auto outside = [&](int i) { return absdist(P.pr[phys(i)].x, usweep) >= df; };
  int lo = 0, hi = 1;
  bool ok1 = false;
  if (act) {
    if (side == 0) { lo = pt.wstart - 1; hi = near; }
    else {
      ok1 = near + 1 <= pt.wend && !outside(near + 1);
      if (ok1) { lo = near + 1; hi = pt.wend + 1; }
    }
  }
  const int e = group_search<G>(lo, hi, lane, [&](int m) { return outside(m) != (side == 1); });
  if (act && (tid & (G - 1)) == 0) {
    Walk& V = S.w[w];
    const int sweep = pt.sweep;
    const double la = W.la;
    if (side == 0) {
      V.len = outside(near) ? 0 : 1;
      V.nl = near - e;
      V.xl = log_ad_of(e < near ? e : near, sweep, la, P);
    } else {
      const int r = ok1 ? e - 1 : near;
      V.nr = r - near;
      V.xr = log_ad_of(r, sweep, la, P);
    }
  }
}

template <class SM>
__device__ __forceinline__ void walk_bounds_par(SM& S, const Params& P, int tid, int nw) {
  if (2 * nw * 16 <= WG) walk_bounds_g<16>(S, P, tid, nw);  // uniform over the workgroup
  else if (2 * nw * 8 <= WG) walk_bounds_g<8>(S, P, tid, nw);
  else walk_bounds_g<4>(S, P, tid, nw);  // split cells' speculative phases (up to 64 walks)
}

// exact sequential sum of one walk by one wave (slow path, settles an argmax), 64 terms at
// a time.  A chunk whose partial sums provably stay inside the binade of the running value
// acc (u = its ulp) and holds no tie adds exactly acc + u * sum(rint(t/u)) (SURVEY Appendix
// B, per chunk): one wave reduction.  Otherwise (a binade edge within reach, a tie, acc >= 0)
// the chunk is added term by term as the reference does.  Walks that leave the binade of the
// window null sum (ascertainment-corrected tables: sums far below null) cross a few binades,
// so almost every chunk takes the reduction.
// acc + t_0 + t_1 + ... + t_{lim-1} in that order, exactly as the sequential fp adds do, for
// one wave whose lane l holds t_l (lanes >= lim hold 0.0): one wave reduction when the chunk
// provably stays in acc's binade with no tie, else term by term
__device__ __forceinline__ double exact_chunk_add(double acc, double t, int lim) {
  {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(acc);
    const int be = (int)((bits >> 52) & 0x7FF);
    if (acc < 0.0 && be > 52 && be < 0x7FF - 52) {
      const double inv = __longlong_as_double((long long)(2098 - be) << 52);   // 2^(52 - e), e = be - 1023
      const double u = __longlong_as_double((long long)(be - 52) << 52);       // 2^(e - 52)
      const double q = t * inv, R = rint(q);
      if (!__any(fabs(q - R) == 0.5) && !__any(!(fabs(R) < 4503599627370496.0))) {  // no tie, |R| < 2^52
        double sp = R > 0.0 ? R : 0.0, sn = R < 0.0 ? R : 0.0;  // |sums| < 2^58: exact only below 2^53,
#pragma unroll                                                  // checked by the bounds below
        for (int o = 32; o > 0; o >>= 1) { sp += __shfl_xor(sp, o, 64); sn += __shfl_xor(sn, o, 64); }
        const double A0 = acc * inv;  // an integer in (-2^53, -2^52]
        // every partial lies in [A0 + sn, A0 + sp]; inside (-2^53, -2^52] it stays in the binade
        if (sp < 9007199254740992.0 && sn > -9007199254740992.0 && A0 + sn > -9007199254740992.0 &&
            A0 + sp <= -4503599627370496.0)
          return (A0 + sp + sn) * u;
      }
    }
  }
  for (int l = 0; l < lim; l++) acc = acc + __shfl(t, l, 64);
  return acc;
}

template <bool LDS, class SM>
__device__ __forceinline__ double walk_sequential(const SM& S, const Walk& W, const Pt& pt, const Params& P, int lane) {
  double acc = pt.N;
  for (int kb = 0; kb < W.len; kb += 64) {
    const int k = kb + lane;
    double t = 0.0;
    if (k < W.len) t = term_dev<LDS>(walk_index(k, pt.nearest, W.nl), pt.sweep, W.la, S, P);
    acc = exact_chunk_add(acc, t, W.len - kb < 64 ? W.len - kb : 64);
    if (acc != acc) break;  // NaN stays NaN through every later add (NaN spline rows, Q15)
  }
  return acc;
}

// FSCLG_SITE_MAJOR (default): a walk's left part is cut on the grid that ENDS at the block holding the
// nearest site (the right part's grid starts at the block after it), so that both grids are the same
// for every walk of a point, and the waves are dealt a phase's segments site-major: slice (j, part) is
// the j-th segment from the nearest site of every walk that reaches it, so the waves working at once
// read the same sites and log-table entries for different alphas (logt(|d|) does not depend on alpha)
// and those reads hit the vector L1.  0: the left grid from the walk's far end, walk-major dealing.
#ifndef FSCLG_FAR_FIRST
#define FSCLG_FAR_FIRST 0  // site-major slices from the farthest inwards (1) or from the nearest SNP outwards (0)
#endif
#ifndef FSCLG_GROUP_TOL
#define FSCLG_GROUP_TOL 2  // a window group takes the following walks whose window base is at most this far below
#endif
#ifndef FSCLG_SITE_MAJOR
#define FSCLG_SITE_MAJOR 1
#endif
#ifndef FSCLG_LEFT_ANCHOR
#define FSCLG_LEFT_ANCHOR FSCLG_SITE_MAJOR
#endif
__device__ __forceinline__ int left_anchor(int near) { return (near & ~127) + 128; }

// A walk covers the site indices [nearest - nl, nearest + nr]; its left part
// [nearest - nl, nearest] (walked downwards, sm-search.c:122-128) and right part
// [nearest + 1, nearest + nr] are cut into separate segments (left ones first), so each
// part's walk order is monotone in the index.  Segments lie on the aligned SEGN-site grid
// that starts at the part's first 128-site block: interior boundaries are trip-aligned, and
// only a part's first and last trips are partial (masked).
template <int SEGN>
__device__ __forceinline__ void seg_bounds(const Walk& W, const Pt& pt, int s, int& ib, int& ie) {
  const int lo = pt.nearest - W.nl, near = pt.nearest, hi = pt.nearest + W.nr;
  if (s < W.nsl) {
#if FSCLG_LEFT_ANCHOR
    const int A = left_anchor(near), j = W.nsl - 1 - s;
    ib = max(lo, A - (j + 1) * SEGN); ie = min(A - j * SEGN, near + 1);
#else
    const int b0 = lo & ~127;
    ib = max(lo, b0 + s * SEGN); ie = min(b0 + (s + 1) * SEGN, near + 1);
#endif
  } else {
    const int b1 = (near + 1) & ~127, t = s - W.nsl;
    ib = max(near + 1, b1 + t * SEGN); ie = min(b1 + (t + 1) * SEGN, hi + 1);
  }
}

// segments of a walk's two parts (layout)
template <int SEGN>
__device__ __forceinline__ void seg_counts(int lo, int near, int hi, int& nsl, int& nsr) {
#if FSCLG_LEFT_ANCHOR
  nsl = (left_anchor(near) - (lo & ~127) + SEGN - 1) / SEGN;
#else
  nsl = (near - (lo & ~127)) / SEGN + 1;
#endif
  nsr = hi > near ? (hi - ((near + 1) & ~127)) / SEGN + 1 : 0;
}


// the segment of site index i of the walk
template <int SEGN>
__device__ __forceinline__ int seg_of(const Walk& W, const Pt& pt, int i) {
  const int lo = pt.nearest - W.nl, near = pt.nearest;
#if FSCLG_LEFT_ANCHOR
  (void)lo;
  return i <= near ? W.nsl - 1 - (left_anchor(near) - 1 - i) / SEGN : W.nsl + (i - ((near + 1) & ~127)) / SEGN;
#else
  return i <= near ? (i - (lo & ~127)) / SEGN : W.nsl + (i - ((near + 1) & ~127)) / SEGN;
#endif
}

__device__ __forceinline__ bool odd_int(double v) { return v - 2.0 * floor(0.5 * v) != 0.0; }

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// a wave-uniform double into scalar registers
__device__ __forceinline__ double uniform_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// FSCLG_TRIP_STAMPS (diagnostic build): per-trip phase times of the term loop, by s_memtime
// stamps (each forces the waits before it): stats[8..23] = trips, then cycles in (nx wait +
// |d|), (log distance + interval test), (coefficients + polynomial), (sums, ties, look-ahead),
// trips per coefficient path (LDS, global, per lane) and the coefficient phase's cycles per
// path, trips per log-distance path (LDS far, global mid, per lane) and the log phase's cycles
// per path
#ifdef FSCLG_TRIP_STAMPS
#define TSTAMP(v) do { __builtin_amdgcn_sched_barrier(0); \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) :: "memory"); \
    __builtin_amdgcn_sched_barrier(0); } while (0)
#endif

// one index-order segment of one walk, by one wave, with a wave-uniform spline interval.  Along a segment
// the sites move monotonically away from (or towards) the sweep, and a trip's 64*U sites
// usually span a small fraction of one interval, so the wave carries the interval civ of its
// last site with its exact bounds [thr[civ], thr[civ+1]) in scalar registers: when every
// lane's x lies inside (two compares per term) the interval is civ for all of them, with no
// per-lane interval arithmetic, and the coefficient block comes from one place (the LDS
// window or the global table, a uniform branch).  Otherwise the trip takes the per-lane path
// of run_segment and re-centres civ on its last site.  Only the final trip of a segment
// masks lanes past its end (zero sentinel row).
template <bool LDS, int SEGN, int U, class SM>
__device__ __forceinline__ void run_segment_idx(SM& S, int w, int s, int s1, const Params& P, int lane,
                                                double& acc, double& accm) {
  const Walk& W = S.w[w];
  const Pt& pt = S.pt[W.p];
  const uint32_t usweep = (uint32_t)pt.sweep ^ POS_BIAS;
  const double la = W.la, inv = pt.inv_u;
  const int lo = pt.nearest - W.nl;
  int ib, ie;
  seg_bounds<SEGN>(W, pt, s, ib, ie);
  // trips run over the aligned 128-site blocks from bs: sites bs + k, k in [k0, n), belong to
  // the segment (lanes outside it take the zero sentinel row)
  int bs = ib & ~127, k0 = ib - bs, n = ie - bs;
  const int ivc0 = __builtin_amdgcn_readfirstlane(S.ivc0);
  const double* thrp = LDS ? reinterpret_cast<const double*>(fsclg_dyn + P.off_thr) : P.thr;
  int civ = 0;
  double sum = 0.0, mag = 0.0;
  // the sites of the next trip are loaded one trip ahead (nx, one dwordx4: sites bs + kb +
  // lane and + 64 + lane of the interleaved array), issued after the trip's own coefficient
  // loads so that waiting for a global coefficient gather (vmcnt counts in order) does not
  // wait for them; PAD covers the look-ahead past a segment's end
  uint4 nx[U / 2];
#pragma unroll
  for (int j = 0; j < U / 2; j++) nx[j] = ld_trip(P.pr, (uint32_t)(bs + 128 * j), lane);
#ifdef FSCLG_TRIP_STAMPS
  unsigned long long tsa[16] = {0};
#endif
  auto trip = [&](const int kb, auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;
#ifdef FSCLG_TRIP_STAMPS
    unsigned long long t_a, t_b, t_c, t_d, t_e;
    int lpath = 2, cpath = 2;
    TSTAMP(t_a);
#endif
    uint32_t pv[U], rv[U];
    bool valid[U];
#pragma unroll
    for (int j = 0; j < U / 2; j++) { pv[2 * j] = nx[j].x; rv[2 * j] = nx[j].y; pv[2 * j + 1] = nx[j].z; rv[2 * j + 1] = nx[j].w; }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int k = kb + 64 * u + lane;
      valid[u] = !MASK || (k >= k0 && k < n);
      if (!valid[u]) rv[u] = 0u;  // zero sentinel row outside the segment
    }
    // log distance: when every lane's |d| lies in the LDS copy of the far branch (one
    // unsigned compare per site: |d| in [2^24, lt_hi << 16)), straight from LDS; when every
    // lane's |d| is in the mid branch, one gather each with no branch select; otherwise per
    // lane (logt_lds).  Every lane is active in a trip, so the wave-wide tests below
    // compare ballots with all ones.
    double x[U];
    uint32_t ad[U];
    bool far = true;
#pragma unroll
    for (int u = 0; u < U; u++) {
      ad[u] = absdist(pv[u], usweep);
      far = far && (ad[u] - 0x1000000u < (uint32_t)P.lt_span);
    }
    bool mid = true;  // every |d| in the mid branch (2^16 <= |d| < 2^24): one global gather each
#pragma unroll
    for (int u = 0; u < U; u++) mid = mid && (ad[u] - 0x10000u < 0xFF0000u);
#ifdef FSCLG_TRIP_STAMPS
    TSTAMP(t_b);
    lpath = (LDS && __builtin_amdgcn_ballot_w64(far) == ~0ull) ? 0 : (__builtin_amdgcn_ballot_w64(mid) == ~0ull ? 1 : 2);
#endif
    if (LDS && __builtin_amdgcn_ballot_w64(far) == ~0ull) {
      const double* lt2 = reinterpret_cast<const double*>(fsclg_dyn + P.off_lt);  // pre-offset by -256 entries
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = lt2[ad[u] >> 16] + la;
    } else if (__builtin_amdgcn_ballot_w64(mid) == ~0ull) {
#if FSCLG_LOG_CALC
      if (LDS && lx_kernel<SM>() && P.lx_on) {
        const double* lx = reinterpret_cast<const double*>(fsclg_dyn + P.off_lx);
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = logx_mid(ad[u] >> 8, lx) + la;
      } else
#endif
      {
        const char* lt1 = reinterpret_cast<const char*>(P.logt3 + 0x10000);
#pragma unroll
        for (int u = 0; u < U; u++) x[u] = *reinterpret_cast<const double*>(lt1 + ((ad[u] >> 8) << 3)) + la;
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = logt_lds<LDS>(ad[u], P) + la;
    }
    if (kb == 0) {  // a segment's first trip: centre the interval on its last site
      const double xl = readlane_f64(x[U - 1], 63);
      civ = __builtin_amdgcn_readfirstlane(interval_of<LDS>(xl, S, P));
    }
    // the bounds of civ, read afresh each trip (a broadcast LDS read): carried across trips
    // they cost four 64-bit register copies per trip at the loop's phi
    const double tlo = thrp[civ], thi = thrp[civ + 1];
    // one ballot per compare (SGPR masks, no bool materialised per lane)
    unsigned long long inm = ~0ull;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if constexpr (MASK) {  // masked lanes add exactly 0 anyway
        const bool ok = ((x[u] >= tlo) && (x[u] < thi)) || !valid[u];
        inm &= __builtin_amdgcn_ballot_w64(ok);
      } else {
        inm &= __builtin_amdgcn_ballot_w64(x[u] >= tlo) & __builtin_amdgcn_ballot_w64(x[u] < thi);
      }
    }
    const bool uni = inm == ~0ull;
    double2 ca[U], cb[U];
#ifdef FSCLG_TRIP_STAMPS
    TSTAMP(t_c);
    cpath = !uni ? 2 : ((LDS && (uint32_t)(civ - ivc0) < (uint32_t)P.n_civ) ? 0 : 1);
#endif
#ifdef FSCLG_PATHSTATS  // diagnostic: trips per path in the stats slots 4 (per-lane), 5 (LDS), 6 (global)
    if (lane == 0) atomicAdd(&S.cnt[!uni ? 4 : ((LDS && (uint32_t)(civ - ivc0) < (uint32_t)P.n_civ) ? 5 : 6)], 1ull);
#endif
    if (uni) {
#ifdef FSCLG_EXP_COEF_LDS
      const uint32_t ci = min((uint32_t)(civ - ivc0), (uint32_t)P.civ_max);
      if (LDS && P.n_civ > 0) {
#else
      const uint32_t ci = (uint32_t)(civ - ivc0);
      if (LDS && ci < (uint32_t)P.n_civ) {
#endif
        const char* lb = fsclg_dyn + (__umul24(ci, (uint32_t)P.stride) << 5);
#pragma unroll
        for (int u = 0; u < U; u++) coef_ld(lb, rv[u] << 4, P, ca[u], cb[u]);
      } else {
        const char* gb = reinterpret_cast<const char*>(P.coef) + (__umul24((uint32_t)civ, (uint32_t)P.stride) << 5);
#pragma unroll
        for (int u = 0; u < U; u++) coef_ld(gb, rv[u] << 4, P, ca[u], cb[u]);
      }
    } else {
      int iv[U];
      coef_stage<LDS, U>(x, rv, S, P, ivc0, ca, cb, iv);
      civ = __builtin_amdgcn_readlane(iv[U - 1], 63);  // the trip's last site
    }
    double nul[U];
#pragma unroll
    for (int u = 0; u < U; u++) nul[u] = null_of<LDS>(rv[u], S, P);
#ifdef FSCLG_EXP_COEF_LDS  // the lanes whose interval missed the window add 0 (sane sums, the same trips)
    bool miss[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      miss[u] = (uint32_t)((uni ? civ : interval_of<LDS>(x[u], S, P)) - ivc0) >= (uint32_t)P.n_civ;
#endif
    // after the last use of this trip's rows (so the look-ahead loads into the same
    // registers, no copy at the loop edge), unconditional (the last trip's look-ahead reads
    // the padding; a conditional load would make the waits below conservative at the join)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < U / 2; j++) nx[j] = ld_trip(P.pr, (uint32_t)(bs + kb + 64 * U + 128 * j), lane);
    __builtin_amdgcn_sched_barrier(0);
#ifdef FSCLG_TRIP_STAMPS
    double yv[U];
#pragma unroll
    for (int u = 0; u < U; u++) yv[u] = x[u] * (ca[u].x * x[u] * x[u] + ca[u].y * x[u] + cb[u].x) + cb[u].y;
    {
      double yy = yv[0];
#pragma unroll
      for (int u = 1; u < U; u++) yy += yv[u];
      asm volatile("" :: "v"(yy));
    }
    TSTAMP(t_d);
#endif
#pragma unroll
    for (int u = 0; u < U; u++) {
#ifdef FSCLG_TRIP_STAMPS
      const double y = yv[u];
#else
      double y = x[u] * (ca[u].x * x[u] * x[u] + ca[u].y * x[u] + cb[u].x) + cb[u].y;
#endif
#ifdef FSCLG_EXP_COEF_LDS
      if (miss[u]) y = nul[u] + 0.0 * y;
#endif
      const double q = (y - nul[u]) * inv;
      const double R = rint(q);                 // the even neighbour at a tie; the resolver settles ties
      const double fr = q - R;
      if (__ballot(fabs(fr) == 0.5)) {          // rare: record the tie with its in-segment prefix parity
        const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const unsigned long long ps = __ballot(odd_int(sum));
        const unsigned long long pr = __ballot(odd_int(R));
        const int pre = (__popcll(ps) + __popcll(pr & below)) & 1;
        if (fabs(fr) == 0.5) {
          const int ti = atomicAdd(&S.n_ties, 1);
          if (ti < MAXTIES)
            S.ties[ti] = (w << 20) | ((fr < 0.0 ? 1 : 0) << 19) | (pre << 18) | (bs + kb + 64 * u + lane - lo);
        }
      }
      sum += R;
      mag += fabs(R);
    }
#ifdef FSCLG_TRIP_STAMPS
    asm volatile("" :: "v"(sum), "v"(mag));
    TSTAMP(t_e);
    tsa[0] += 1; tsa[1] += t_b - t_a; tsa[2] += t_c - t_b; tsa[3] += t_d - t_c; tsa[4] += t_e - t_d;
    tsa[5 + cpath] += 1; tsa[8 + cpath] += t_d - t_c; tsa[11 + lpath] += 1;
    if (lpath == 1) tsa[14] += t_c - t_b; else if (lpath == 0) tsa[15] += t_c - t_b;
#endif
  };
  for (;;) {
    int kb = 0;
    if (k0 > 0) { trip(0, std::true_type{}); kb = 64 * U; }  // a part's first trip starts mid-block
    for (; kb + 64 * U <= n; kb += 64 * U) trip(kb, std::false_type{});
    if (kb < n) trip(kb, std::true_type{});
    const unsigned long long odd = __ballot(odd_int(sum));
    if (lane == 0 && (__popcll(odd) & 1)) atomicXor(&S.segbits[w][s >> 5], 1u << (s & 31));
#ifdef FSCLG_TRIP_STAMPS
    if (lane == 0)
      for (int j = 0; j < 16; j++) atomicAdd(P.stats + 8 + j, tsa[j]);
    for (int j = 0; j < 16; j++) tsa[j] = 0;
#endif
    acc += sum;
    accm += mag;
    if (++s >= s1) break;
    seg_bounds<SEGN>(W, pt, s, ib, ie);
    bs = ib & ~127; k0 = ib - bs; n = ie - bs;
#pragma unroll
    for (int j = 0; j < U / 2; j++) nx[j] = ld_trip(P.pr, (uint32_t)(bs + 128 * j), lane);
    sum = 0.0; mag = 0.0;
  }
}

// a wave's share of walk w: int64 totals of sum R and sum |R| into S.P / S.Q.  Exact when
// every lane's |R| total is below 2^51 (then all fp64 partials were exact, fl being
// monotone; NaN fails the test); 8 waves x 64 lanes keep the walk's totals below 2^60.
template <class SM>
__device__ __forceinline__ void flush_walk(SM& S, int w, double acc, double accm, int lane) {
  const bool big = !(accm < 2251799813685248.0);  // 2^51
  const long long isum = wave_sum64(big ? 0 : (long long)acc);
  const long long imag = wave_sum64(big ? 0 : (long long)accm);
  const bool anybig = __any(big);
  if (lane == 0) {
    atomicAdd(&S.P[w], (unsigned long long)isum);
    atomicAdd(&S.Q[w], (unsigned long long)imag);
  }
  if (anybig) {  // rare (terms near log(DBL_MIN) of ascertainment-corrected tables): approximate sums
    double da = big ? acc : 0.0, dm = big ? accm : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { da += __shfl_xor(da, o, 64); dm += __shfl_xor(dm, o, 64); }
    if (lane == 0) {
      atomicAdd(&S.Pd[w], da);
      atomicAdd(&S.Qd[w], dm);
      atomicOr(&S.wflag[w], 1);
    }
  }
}

// resolve walk w's exact value (thread per walk).  S.P = sum R, S.Q = sum |R| over the walk.
// Ties are replayed in k order: fl(acc + t) rounds to even, so where t/u = F + 1/2 an odd
// running sum takes the other neighbour of the even R (+1 if R = F, -1 if R = F + 1).
template <int SEGN, bool BAND = false, class SM>
__device__ __forceinline__ void resolve_walk(SM& S, int w) {
  constexpr int WM = BAND ? 31 : 63;  // band mode: walk in bits 20-24, the tie's segment in bits 25-31
  const Walk& W = S.w[w];
  const Pt& pt = S.pt[W.p];
  if (W.len == 0) { S.exact[w] = 1; S.val[w] = pt.N; return; }
  const long long Ssum = (long long)S.P[w], A = (long long)S.Q[w];
  const long long Pp = (Ssum + A) / 2, Qn = (Ssum - A) / 2;   // positive / negative parts
  const bool overflow = S.n_ties > MAXTIES;
  int T = 0;
  const int nt = S.n_ties < MAXTIES ? S.n_ties : MAXTIES;
  for (int j = 0; j < nt; j++) T += (((S.ties[j] >> 20) & WM) == w);
  const bool big = S.wflag[w] != 0 || pt.inv_u == 0.0;
  const long long S0 = pt.inv_u == 0.0 ? 0 : (long long)(pt.N * pt.inv_u);
  const long long LO = -(1ll << 53), HI = -((1ll << 52) + 1);
  const bool safe = !big && !overflow && S0 < 0 && (S0 + Qn - T >= LO) && (S0 + Pp + T <= HI);
  if (safe) {
    const int nl = W.nl, nsl = W.nsl;
    auto segpar = [&](int a, int b) {  // parity of the segment bits [a, b)
      int par = 0;
      for (int j = a >> 5; j <= (b - 1) >> 5 && a < b; j++) {
        unsigned int m = S.segbits[w][j];
        if (j == a >> 5) m &= ~0u << (a & 31);
        if (j == (b - 1) >> 5 && (b & 31)) m &= ~0u >> (32 - (b & 31));
        par ^= __popc(m) & 1;
      }
      return par;
    };
    const int lpar = segpar(0, nsl);
    int adjx = 0;
    long long adjs = 0;
    int prevk = -1;
    for (int c = 0; c < T; c++) {  // ties of this walk in k order
      int bestk = 0x7fffffff, bestv = 0;
      for (int j = 0; j < nt; j++) {
        const int v = S.ties[j];
        const int jj = v & 0x3FFFF;
        const int k = jj <= nl ? nl - jj : jj;
        if (((v >> 20) & WM) == w && k > prevk && k < bestk) { bestk = k; bestv = v; }
      }
      prevk = bestk;
      // parity of the running sum before this term: S0, then the terms before it in k
      // order = (left tie) the left part after it, (right tie) the left part and the
      // right part before it; R of a tie is even, so both read lpar ^ prefix-in-part
      const int jj = bestv & 0x3FFFF;
      const int sg = BAND ? (int)((unsigned)bestv >> 25) : seg_of<SEGN>(W, pt, pt.nearest - nl + jj);
      const int sp = segpar(jj <= nl ? 0 : nsl, sg);
      const int pre = (bestv >> 18) & 1, up = (bestv >> 19) & 1;
      const int adj = (int)(S0 & 1) ^ lpar ^ sp ^ pre ^ adjx;
      adjx ^= adj;
      adjs += adj ? (up ? -1 : 1) : 0;
    }
    S.exact[w] = 1;
    S.val[w] = (double)(S0 + Ssum + adjs) * pt.u;
  } else {
    S.exact[w] = 0;
    if (pt.inv_u == 0.0) {
      S.appr[w] = __longlong_as_double(0x7FF0000000000000ll);  // unknown: forces the slow path if it matters
      S.bnd[w] = 0.0;
    } else if (big) {
      // some lanes' fp64 accumulators passed 2^51: their sums are approximate, each off by at
      // most (terms summed) * 2^-53 * (their sum of |R|), and so is every later add (wave tree,
      // LDS atomics); the reference's own sequential rounding and the per-term rint as below
      const double u = pt.u, len = (double)W.len;
      const double qt = (double)A + S.Qd[w];
      const double smax = fabs(pt.N) + (qt + len) * u;
      S.appr[w] = pt.N + ((double)Ssum + S.Pd[w]) * u;
      S.bnd[w] = 2.0 * (len * u + len * 4.440892098500626e-16 * smax) + 2.0 * (len + 256.0) * 2.220446049250313e-16 * qt * u +
                 1e-300;
      // a NaN sum has a NaN term (R = rint(t/u) is finite for finite t) or both infinities
      // among the terms: the sequential sum of sm-search.c is then NaN in any order, and a
      // NaN never wins the strict '>' of search_maxalpha (NaN spline rows, Q15)
      if (S.appr[w] != S.appr[w]) { S.exact[w] = 1; S.val[w] = S.appr[w]; }
    } else {
      const double u = pt.u, len = (double)W.len;
      const double smax = fabs(pt.N) + ((double)A + len) * u;
      S.appr[w] = (double)(S0 + Ssum) * u;
      S.bnd[w] = 2.0 * (len * u + len * 4.440892098500626e-16 * smax) + 1e-300;
    }
    atomicAdd(&S.cnt[4], 1ull);
  }
}

// evaluate S.nwalk walks (already holding p, la) -> exact values in S.val
// stage the coefficient blocks of intervals [wb, wb + n_civ) x every row into LDS, in the
// table's own [iv][row][4] layout: one contiguous copy (all threads; the caller brackets
// it with barriers)
template <class SM>
__device__ __forceinline__ void load_window(SM& S, const Params& P, int wb) {
  double2* dst = reinterpret_cast<double2*>(fsclg_dyn);
  const double2* src = reinterpret_cast<const double2*>(P.coef) + (size_t)wb * P.stride * 2;
  for (int e = threadIdx.x; e < 2 * P.n_cache; e += WG) dst[e] = src[e];
  if (threadIdx.x == 0) S.ivc0 = wb;
}

// ------------------------------------------------------------ band mode
constexpr int TPS = SEG / 128;           // trips per segment (band mode)
constexpr uint32_t DNONE = 0xFFFFFFFFu;  // no lazy cut on that trip (|d| never reaches it)
static_assert(U_MAIN == 2, "band mode: one aligned 128-site block per trip");
static_assert(MAXWALK <= 32, "band mode: the walk in 5 bits of a tie record");

// piece q of walk w (q in site-index order, BandLds): its part, trip range [ta, tb] relative to
// the part's first trip, and its lazy cuts (the band whose |d| bound is tested on the first /
// last trip; -1: none).  Left part (walked downwards): q = band, q = nb the remainder next to the
// nearest site; a site of band b lies in (cut(b - 1), cut(b)] where cut(x) is the LAST site in
// index order with |d| >= D(x).  Right part: q = nb + 1 the remainder, then bands nb - 1 .. 0; a
// site of band b lies in [cut(b), cut(b - 1)) with cut(x) the FIRST site with |d| >= D(x).
struct Piece { int part, ta, tb, clo, chi; bool empty; };
// a walk part's cuts in registers (one 16-byte LDS read); element access by unrolled selects
static_assert(NBMAX == 8, "a part's cuts are one 16-byte LDS word");
struct Cuts { int c[NBMAX]; };
__device__ __forceinline__ Cuts load_cuts(const BandLds& bd, int w, int part) {
  const uint4 v = *reinterpret_cast<const uint4*>(&bd.cut[w][part][0]);
  const uint32_t a[4] = {v.x, v.y, v.z, v.w};
  Cuts k;
#pragma unroll
  for (int i = 0; i < 4; i++) { k.c[2 * i] = (int)(int16_t)(a[i] & 0xFFFFu); k.c[2 * i + 1] = (int)(int16_t)(a[i] >> 16); }
  return k;
}
__device__ __forceinline__ void store_cuts(BandLds& bd, int w, int part, const Cuts& k) {
  uint32_t a[4];
#pragma unroll
  for (int i = 0; i < 4; i++) a[i] = ((uint32_t)k.c[2 * i] & 0xFFFFu) | ((uint32_t)k.c[2 * i + 1] << 16);
  *reinterpret_cast<uint4*>(&bd.cut[w][part][0]) = make_uint4(a[0], a[1], a[2], a[3]);
}
__device__ __forceinline__ int cut_at(const Cuts& k, int i) {  // k.c[i], i in [0, NBMAX)
  int v = -1;
#pragma unroll
  for (int j = 0; j < NBMAX; j++) if (j == i) v = k.c[j];
  return v;
}
__device__ __forceinline__ int kept_below(const Cuts& k, int b) {  // the largest j < b with a kept cut, -1
  int f = -1;
#pragma unroll
  for (int j = 0; j < NBMAX; j++) if (j < b && k.c[j] >= 0) f = j;
  return f;
}
// piece q of a walk (site-index order, BandLds) from its part's cuts k: left part (q <= nb): band q,
// q = nb the remainder, the piece ending (inclusive) at its own kept cut and starting past the
// nearest kept cut of a higher band; right part: q = nb + 1 the remainder, then bands nb - 1 .. 0,
// the piece starting at its own kept cut and ending before the nearest kept cut of a higher band
__device__ __forceinline__ Piece piece_of(const Cuts& k, int q, int nb, int ntrL, int ntrR) {
  Piece pc;
  pc.clo = -1; pc.chi = -1; pc.empty = false;
  if (q <= nb) {
    const int b = q;
    pc.part = 0; pc.ta = 0; pc.tb = ntrL - 1;
    const int f = kept_below(k, b);
    if (f >= 0) { pc.ta = cut_at(k, f); pc.clo = f; }
    if (b < nb) {
      const int c = cut_at(k, b);
      if (c < 0) pc.empty = true;
      else { pc.tb = c; pc.chi = b; }
    }
    if (ntrL <= 0) pc.empty = true;
  } else {
    const int b = nb - (q - nb - 1);
    pc.part = 1; pc.ta = 0; pc.tb = ntrR - 1;
    if (b < nb) {
      const int c = cut_at(k, b);
      if (c < 0) pc.empty = true;
      else { pc.ta = c; pc.clo = b; }
    }
    const int f = kept_below(k, b);
    if (f >= 0) { pc.tb = cut_at(k, f); pc.chi = f; }
    if (ntrR <= 0) pc.empty = true;
  }
  return pc;
}

// trips of the two parts of walk w (0 when the walk is empty)
template <class SM>
__device__ __forceinline__ void part_trips(const SM& S, int w, int& ntrL, int& ntrR) {
  const Walk& W = S.w[w];
  const int near = S.pt[W.p].nearest;
  ntrL = W.len ? (near >> 7) - ((near - W.nl) >> 7) + 1 : 0;
  ntrR = W.len && W.nr > 0 ? ((near + W.nr) >> 7) - ((near + 1) >> 7) + 1 : 0;
}

__device__ __forceinline__ int first_set128(unsigned long long b0, unsigned long long b1) {
  return b0 ? __ffsll(b0) - 1 : (b1 ? 64 + __ffsll(b1) - 1 : 128);
}
__device__ __forceinline__ int last_set128(unsigned long long b0, unsigned long long b1) {
  return b1 ? 127 - __clzll(b1) : (b0 ? 63 - __clzll(b0) : -1);
}

// one segment of one piece by one wave: nt trips from block t0 (absolute), the part's site range
// masking its first and last trips, and the piece's lazy cuts (thresholds dlo on the first trip,
// dhi on the last; DNONE: none) masking the boundary trips it shares with its neighbours.  A
// lazy cut is a function of the trip's sites alone (a ballot of |d| >= D over the part's sites of
// the trip), so the two pieces on either side of it split that trip's sites exactly between them,
// whatever the data.  Otherwise as run_segment_idx, whose trip this is.
template <bool LDS, class SM>
__device__ __forceinline__ void run_piece_seg(SM& S, int w, int part, int sid, int t0, int nt, uint32_t dlo,
                                              uint32_t dhi, const Params& P, int lane, double& acc, double& accm) {
  constexpr int U = 2;
  const Walk& W = S.w[w];
  const Pt& pt = S.pt[W.p];
  const uint32_t usweep = (uint32_t)pt.sweep ^ POS_BIAS;
  const double la = W.la, inv = pt.inv_u;
  const int lo = pt.nearest - W.nl;
  const int plo = part ? pt.nearest + 1 : lo, phi = part ? pt.nearest + W.nr : pt.nearest;
  const int ivc0 = __builtin_amdgcn_readfirstlane(S.ivc0);
  const double* thrp = LDS ? reinterpret_cast<const double*>(fsclg_dyn + P.off_thr) : P.thr;
  const int bs0 = t0 << 7;
  int civ = 0;
  double sum = 0.0, mag = 0.0;
  uint4 nx = ld_trip(P.pr, (uint32_t)bs0, lane);
  auto trip = [&](const int bs, const bool first, const bool lzlo, const bool lzhi, auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;
    uint32_t pv[U], rv[U], ad[U];
    bool valid[U];
    pv[0] = nx.x; rv[0] = nx.y; pv[1] = nx.z; rv[1] = nx.w;
#pragma unroll
    for (int u = 0; u < U; u++) ad[u] = absdist(pv[u], usweep);
    if constexpr (MASK) {
      int kmin = max(plo - bs, 0), kmax = min(phi - bs, 127);
      const bool in0 = lane >= kmin && lane <= kmax, in1 = lane + 64 >= kmin && lane + 64 <= kmax;
      if (lzlo) {
        const unsigned long long b0 = __ballot(in0 && ad[0] >= dlo), b1 = __ballot(in1 && ad[1] >= dlo);
        kmin = max(kmin, part ? first_set128(b0, b1) : last_set128(b0, b1) + 1);
      }
      if (lzhi) {
        const unsigned long long b0 = __ballot(in0 && ad[0] >= dhi), b1 = __ballot(in1 && ad[1] >= dhi);
        kmax = min(kmax, part ? first_set128(b0, b1) - 1 : last_set128(b0, b1));
      }
      valid[0] = lane >= kmin && lane <= kmax;
      valid[1] = lane + 64 >= kmin && lane + 64 <= kmax;
#pragma unroll
      for (int u = 0; u < U; u++) if (!valid[u]) rv[u] = 0u;  // zero sentinel row
    } else {
      valid[0] = valid[1] = true;
    }
    double x[U];
    bool far = true, mid = true;
#pragma unroll
    for (int u = 0; u < U; u++) {
      far = far && (ad[u] - 0x1000000u < (uint32_t)P.lt_span);
      mid = mid && (ad[u] - 0x10000u < 0xFF0000u);
    }
    if (LDS && __builtin_amdgcn_ballot_w64(far) == ~0ull) {
      const double* lt2 = reinterpret_cast<const double*>(fsclg_dyn + P.off_lt);
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = lt2[ad[u] >> 16] + la;
    } else if (__builtin_amdgcn_ballot_w64(mid) == ~0ull) {
      const char* lt1 = reinterpret_cast<const char*>(P.logt3 + 0x10000);
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = *reinterpret_cast<const double*>(lt1 + ((ad[u] >> 8) << 3)) + la;
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = logt_lds<LDS>(ad[u], P) + la;
    }
    if (first) civ = __builtin_amdgcn_readfirstlane(interval_of<LDS>(readlane_f64(x[U - 1], 63), S, P));
    const double tlo = thrp[civ], thi = thrp[civ + 1];
    unsigned long long inm = ~0ull;
#pragma unroll
    for (int u = 0; u < U; u++) {
      if constexpr (MASK) {
        const bool ok = ((x[u] >= tlo) && (x[u] < thi)) || !valid[u];
        inm &= __builtin_amdgcn_ballot_w64(ok);
      } else {
        inm &= __builtin_amdgcn_ballot_w64(x[u] >= tlo) & __builtin_amdgcn_ballot_w64(x[u] < thi);
      }
    }
    const bool uni = inm == ~0ull;
#ifdef FSCLG_PATHSTATS  // diagnostic: trips per path in the stats slots 4 (per-lane), 5 (LDS), 6 (global)
    if (lane == 0) atomicAdd(&S.cnt[!uni ? 4 : ((LDS && (uint32_t)(civ - ivc0) < (uint32_t)P.n_civ) ? 5 : 6)], 1ull);
#endif
    double2 ca[U], cb[U];
    if (uni) {
      const uint32_t ci = (uint32_t)(civ - ivc0);
      if (LDS && ci < (uint32_t)P.n_civ) {
        const char* lb = fsclg_dyn + (__umul24(ci, (uint32_t)P.stride) << 5);
#pragma unroll
        for (int u = 0; u < U; u++) coef_ld(lb, rv[u] << 4, P, ca[u], cb[u]);
      } else {
        const char* gb = reinterpret_cast<const char*>(P.coef) + (__umul24((uint32_t)civ, (uint32_t)P.stride) << 5);
#pragma unroll
        for (int u = 0; u < U; u++) coef_ld(gb, rv[u] << 4, P, ca[u], cb[u]);
      }
    } else {
      int iv[U];
      coef_stage<LDS, U>(x, rv, S, P, ivc0, ca, cb, iv);
      civ = __builtin_amdgcn_readlane(iv[U - 1], 63);
    }
    double nul[U];
#pragma unroll
    for (int u = 0; u < U; u++) nul[u] = null_of<LDS>(rv[u], S, P);
    __builtin_amdgcn_sched_barrier(0);
    nx = ld_trip(P.pr, (uint32_t)(bs + 128), lane);  // the next trip's sites (PAD covers the last look-ahead)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const double y = x[u] * (ca[u].x * x[u] * x[u] + ca[u].y * x[u] + cb[u].x) + cb[u].y;
      const double q = (y - nul[u]) * inv;
      const double R = rint(q);
      const double fr = q - R;
      if (__ballot(fabs(fr) == 0.5)) {
        const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const unsigned long long ps = __ballot(odd_int(sum));
        const unsigned long long pr = __ballot(odd_int(R));
        const int pre = (__popcll(ps) + __popcll(pr & below)) & 1;
        if (fabs(fr) == 0.5) {
          const int ti = atomicAdd(&S.n_ties, 1);
          if (ti < MAXTIES)
            S.ties[ti] = (int)(((unsigned)sid << 25) | ((unsigned)w << 20) | ((fr < 0.0 ? 1u : 0u) << 19) |
                               ((unsigned)pre << 18) | (unsigned)(bs + 64 * u + lane - lo));
        }
      }
      sum += R;
      mag += fabs(R);
    }
  };
  // the masked trips (a lazy cut, or the part's own first / last block) can only be the first and
  // the last: peeled off, so that the loop body is the unmasked trip alone (a join of both kinds in
  // the loop makes the waits for the look-ahead load conservative: measured 1.7x per trip)
  const bool m0 = dlo != DNONE || bs0 < plo || (nt == 1 && (dhi != DNONE || bs0 + 127 > phi));
  const int bl = bs0 + 128 * (nt - 1);
  const bool ml = nt > 1 && (dhi != DNONE || bl + 127 > phi);
  int t = 0;
  if (m0) { trip(bs0, true, dlo != DNONE, nt == 1 && dhi != DNONE, std::true_type{}); t = 1; }
  const int tend = ml ? nt - 1 : nt;
  for (; t < tend; t++) trip(bs0 + 128 * t, t == 0, false, false, std::false_type{});
  if (ml) trip(bl, false, false, dhi != DNONE, std::true_type{});
  const unsigned long long odd = __ballot(odd_int(sum));
  if (lane == 0 && (__popcll(odd) & 1)) atomicXor(&S.segbits[w][sid >> 5], 1u << (sid & 31));
  acc += sum;
  accm += mag;
}

// the last t in (lo, hi) whose first position is <= key (STRICT: < key), lo if none (positions
// ascend over (lo, hi)): an 8-ary search, seven independent probes per dependent round
template <bool STRICT>
__device__ __forceinline__ int tpos_search(const int32_t* __restrict__ tpos, int lo, int hi, long long key) {
  while (hi - lo > 1) {
    const long long span = hi - lo;
    int m[7];
    bool ok[7];
#pragma unroll
    for (int k = 0; k < 7; k++) m[k] = lo + (int)((span * (k + 1)) >> 3);
#pragma unroll
    for (int k = 0; k < 7; k++) { const long long v = tpos[m[k]]; ok[k] = STRICT ? v < key : v <= key; }
    int nlo = lo, nhi = hi;
#pragma unroll
    for (int k = 0; k < 7; k++)
      if (m[k] > lo && m[k] < hi) {
        if (ok[k]) nlo = max(nlo, m[k]);
        else nhi = min(nhi, m[k]);
      }
    lo = nlo; hi = nhi;
  }
  return lo;
}

// the |d| bound of band b for walk w (band b's sites: |d| >= it)
__device__ __forceinline__ uint32_t band_d(const BandLds& bd, int w, int b) {
  return bd.dv[w][b];
}

// eval_walks in band mode: bounds, the bands and their cuts, the segment numbering, then the
// groups band by band (a "run" stages one band's window and may carry the following bands whose
// pieces are too few to pay for their own), the remainder last; resolve as eval_walks.
template <bool LDS, class SM>
__device__ __forceinline__ void eval_walks_band(SM& S, const Params& P) {
  BandLds& bd = *reinterpret_cast<BandLds*>(fsclg_dyn + P.off_bd);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = __builtin_amdgcn_readfirstlane(S.nwalk);
#ifdef FSCLG_PHASE_TIMING
  unsigned long long t0 = 0;
  if (tid == 0) t0 = wall_clock64();
#define PHASE_MARK(k) do { if (tid == 0) { const unsigned long long t1 = wall_clock64(); S.tph[k] += t1 - t0; t0 = t1; } } while (0)
#else
#define PHASE_MARK(k) do { } while (0)
#endif
  walk_bounds_par(S, P, tid, nw);
  if (tid < nw) {
    S.P[tid] = 0; S.Q[tid] = 0; S.Pd[tid] = 0.0; S.Qd[tid] = 0.0; S.wflag[tid] = 0; S.need_slow[tid] = 0;
    for (int j = 0; j < SEGWORDS; j++) S.segbits[tid][j] = 0;
  }
  if (tid <= NBMAX) { bd.gitems[tid] = 0; bd.gtrips[tid] = 0; }
  if (tid == 0) S.n_ties = 0;
  __syncthreads();
  // the bands: K-interval windows from the phase's top interval T downwards (wave 0, a lane per walk)
  if (wave == 0) {
    const int K = P.n_civ;
    const bool act = lane < nw;
    int len = 0, top = -1;
    if (act) {
      Walk& W = S.w[lane];
      len = W.len ? 1 + W.nl + W.nr : 0;
      W.len = len;
      if (len) top = interval_of<LDS>(fmax(W.xl, W.xr), S, P);
    }
    int T = top;
    long long terms = len;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { T = max(T, __shfl_xor(T, o, 64)); terms += __shfl_xor(terms, o, 64); }
    if (lane == 0) {
      int nb = 0;
      if (T >= 0)
        while (nb < min(P.band_nb, NBMAX)) {
          const int base = T - K * (nb + 1) + 1;
          bd.bbase[nb++] = max(base, 0);
          if (base <= 0) break;
        }
      bd.nb = nb;
      S.cnt[0] += (unsigned long long)terms;
      S.cnt[2] += nw;
    }
  }
  __syncthreads();
  const int nb = __builtin_amdgcn_readfirstlane(bd.nb);
  // the cuts (a thread per walk, part, band): the trip holding the part's first site in walk order
  // whose |d| reaches the band, by bisection over the trips' first positions (sorted within the
  // part; the part's first trip counts as at or before the cut); -1 if the part's farthest site
  // (its largest |d|) stays below the band
  {
    const double* thrp = LDS ? reinterpret_cast<const double*>(fsclg_dyn + P.off_thr) : P.thr;
    for (int it = tid; it < nw * 2 * nb; it += WG) {
      const int w = it / (2 * nb), part = (it / nb) & 1, b = it % nb;
      const Walk& W = S.w[w];
      const Pt& pt = S.pt[W.p];
      const int near = pt.nearest;
      int c = -1;
      if (W.len && (part == 0 || W.nr > 0) && (part ? W.xr : W.xl) >= thrp[bd.bbase[b]]) {
        const uint32_t dvb = P.dband[(size_t)W.kd * (size_t)P.nd + (size_t)bd.bbase[b]];
        bd.dv[w][b] = dvb;
        const long long D = (long long)dvb;
        const long long sw = pt.sweep;
        int t0, lo, hi;
        if (part == 0) {  // the last trip whose first site has pos <= sweep - D
          t0 = (near - W.nl) >> 7;
          lo = t0; hi = (near >> 7) + 1;
          const long long Y = sw - D;
          lo = tpos_search<false>(P.tpos, lo, hi, Y);
        } else {          // the last trip whose first site has pos < sweep + D
          t0 = (near + 1) >> 7;
          lo = t0; hi = ((near + W.nr) >> 7) + 1;
          const long long X = sw + D;
          lo = tpos_search<true>(P.tpos, lo, hi, X);
        }
        c = lo - t0;
      }
      bd.cut[w][part][b] = (int16_t)c;
    }
  }
  __syncthreads();
  // merging, segment numbering and groups (a lane per walk, the walk's cuts in registers).  A cut is
  // kept only where the pieces on both sides hold at least band_minp trips (small pieces cost a
  // segment's fixed work and a masked trip each: 4.8x the segments of the walk-window path with
  // every cut kept); a merged piece goes to the group of its band with the most trips
  if (wave == 0) {
    const bool act = lane < nw && S.w[lane < nw ? lane : 0].len;
    int ntrL = 0, ntrR = 0;
    if (lane < nw) part_trips(S, lane, ntrL, ntrR);
    const int minp = P.band_minp;
    int8_t qL[NBMAX + 1], qR[NBMAX + 1];  // the piece each group processes, per part
#pragma unroll
    for (int g = 0; g <= NBMAX; g++) { qL[g] = -1; qR[g] = -1; }
    Cuts cl = load_cuts(bd, lane < nw ? lane : 0, 0), cr = load_cuts(bd, lane < nw ? lane : 0, 1);
    if (act) {
      // left part, index order: band 0, 1, ..., nb - 1, the remainder; piece b = (cut[b - 1], cut[b]]
      int tr[NBMAX + 1];
      int prev = -1;
#pragma unroll
      for (int b = 0; b <= NBMAX; b++) {
        tr[b] = 0;
        if (b <= nb) {
          const int e = b < NBMAX && b < nb ? cl.c[b < NBMAX ? b : 0] : ntrL - 1;
          if (e >= 0) { tr[b] = e - prev; prev = e; }
        }
      }
      int last = -1, best = nb, btr = -1;
#pragma unroll
      for (int b = 0; b <= NBMAX; b++) {
        if (b <= nb && tr[b] > btr) { btr = tr[b]; best = b; }
        if (b < nb && b < NBMAX) {
          const int c = cl.c[b < NBMAX ? b : 0];
          if (c >= 0) {
            if (c - last >= minp && ntrL - 1 - c >= minp) {
#pragma unroll
              for (int g = 0; g <= NBMAX; g++) if (g == best) qL[g] = (int8_t)b;
              last = c; best = nb; btr = -1;
            } else {
              cl.c[b < NBMAX ? b : 0] = -2;
            }
          }
        } else if (b == nb) {
#pragma unroll
          for (int g = 0; g <= NBMAX; g++) if (g == best) qL[g] = (int8_t)nb;
        }
      }
    }
    if (act && ntrR > 0) {
      // right part, index order: the remainder, band nb - 1, ..., band 0; piece b = [cut[b], cut[b - 1])
      int tr[NBMAX];
      int nxt = ntrR;  // the start of the nearest reached band above
#pragma unroll
      for (int b = 0; b < NBMAX; b++) {
        tr[b] = 0;
        if (b < nb && cr.c[b] >= 0) { tr[b] = nxt - cr.c[b]; nxt = cr.c[b]; }
      }
      int last = 0, low = nb, best = nb, btr = nxt;  // the remainder: [0, lowest reached cut)
#pragma unroll
      for (int k = NBMAX - 1; k >= 0; k--) {  // from the bottom band up
        if (k < nb && cr.c[k] >= 0) {
          const int c = cr.c[k];
          if (c - last >= minp && ntrR - c >= minp) {
#pragma unroll
            for (int g = 0; g <= NBMAX; g++) if (g == best) qR[g] = (int8_t)(nb + 1 + (nb - low));
            last = c; low = k; best = k; btr = tr[k];
          } else {
            cr.c[k] = -2;
            if (tr[k] > btr) { btr = tr[k]; best = k; }
          }
        }
      }
#pragma unroll
      for (int g = 0; g <= NBMAX; g++) if (g == best) qR[g] = (int8_t)(nb + 1 + (nb - low));
    }
    if (lane < nw) {
      store_cuts(bd, lane, 0, cl);
      store_cuts(bd, lane, 1, cr);
#pragma unroll
      for (int g = 0; g <= NBMAX; g++) { bd.qof[lane][0][g] = qL[g]; bd.qof[lane][1][g] = qR[g]; }
    }
    // segment ids in site-index order; each group's segments and trips (LDS atomics)
    int run = 0;
    for (int q = 0; q < 2 * (nb + 1); q++) {
      int nseg = 0;
      if (act) {
        const Piece pc = piece_of(q <= nb ? cl : cr, q, nb, ntrL, ntrR);
        if (!pc.empty && pc.tb >= pc.ta) {
          nseg = (pc.tb - pc.ta + TPS) / TPS;
          int g = -1;
#pragma unroll
          for (int j = 0; j <= NBMAX; j++) if ((q <= nb ? qL[j] : qR[j]) == q) g = j;
          if (g >= 0) { atomicAdd(&bd.gitems[g], nseg); atomicAdd(&bd.gtrips[g], pc.tb - pc.ta + 1); }
        }
      }
      if (lane < nw) bd.sb[lane][q] = (uint8_t)run;
      run += nseg;
    }
    if (lane < nw) {
      bd.sb[lane][2 * (nb + 1)] = (uint8_t)run;
      S.w[lane].nsl = bd.sb[lane][nb + 1];
      S.w[lane].nseg = run;
    }
  }
  __syncthreads();
  if (tid == 0) {  // runs: a band of at least band_th trips stages its window; the rest ride along
      int nr = 0;
      for (int g = 0; g <= nb; g++) {
        const bool st = g < nb && bd.gtrips[g] >= P.band_th;
        if (st || nr == 0) { bd.run_g0[nr] = g; bd.run_stage[nr] = st ? 1 : 0; nr++; }
      }
      bd.run_g0[nr] = nb + 1;
      bd.nrun = nr;
  }
  __syncthreads();
  PHASE_MARK(0);
  {
    int cw = -1;
    double acc = 0.0, accm = 0.0;
    const int nrun = __builtin_amdgcn_readfirstlane(bd.nrun);
    for (int r = 0; r < nrun; r++) {
      const int g0 = __builtin_amdgcn_readfirstlane(bd.run_g0[r]), g1 = __builtin_amdgcn_readfirstlane(bd.run_g0[r + 1]);
      if (__builtin_amdgcn_readfirstlane(bd.run_stage[r])) {
        const int wb = __builtin_amdgcn_readfirstlane(bd.bbase[g0]);
        if (wb != __builtin_amdgcn_readfirstlane(S.ivc0)) {  // uniform over the workgroup
          __syncthreads();
          load_window(S, P, wb);
          __syncthreads();
        }
      }
      int nit = 0;
      for (int g = g0; g < g1; g++) nit += __builtin_amdgcn_readfirstlane(bd.gitems[g]);
      // each wave takes a contiguous run of the items (consecutive items are mostly one walk's: one
      // flush per walk, not per item)
      int g = g0, e = 0, ebase = 0;  // entry e = (walk e >> 1, part e & 1) of group g: items from ebase
      const int i1 = (nit * (wave + 1)) / NWAVE;
      for (int i = (nit * wave) / NWAVE; i < i1; i++) {
        int q, cnt;
        for (;;) {
          const int w = e >> 1, part = e & 1;
          q = bd.qof[w][part][g];
          cnt = q >= 0 ? (int)bd.sb[w][q + 1] - (int)bd.sb[w][q] : 0;
          if (i < ebase + cnt) break;
          ebase += cnt;
          if (++e == 2 * nw) { e = 0; g++; }
        }
        const int w = e >> 1, part = e & 1, s = i - ebase;
        const int sid = (int)bd.sb[w][q] + s;
        int ntrL, ntrR;
        part_trips(S, w, ntrL, ntrR);
        const Piece pc = piece_of(load_cuts(bd, w, part), q, nb, ntrL, ntrR);
        const Walk& W = S.w[w];
        const int near = S.pt[W.p].nearest;
        const int ts = pc.ta + s * TPS, nt = min(TPS, pc.tb - ts + 1);
        const uint32_t dlo = (s == 0 && pc.clo >= 0) ? band_d(bd, w, pc.clo) : DNONE;
        const uint32_t dhi = (ts + nt - 1 == pc.tb && pc.chi >= 0) ? band_d(bd, w, pc.chi) : DNONE;
        const int tp0 = part ? (near + 1) >> 7 : (near - W.nl) >> 7;
        if (w != cw) {
          if (cw >= 0) flush_walk(S, cw, acc, accm, lane);
          cw = w; acc = 0.0; accm = 0.0;
        }
#ifdef FSCLG_SEGSTATS  // diagnostic: segments in the stats slot 6 (n_ties)
        if (lane == 0) atomicAdd(&S.cnt[6], 1ull);
#endif
        run_piece_seg<LDS>(S, w, part, sid, tp0 + ts, nt, dlo, dhi, P, lane, acc, accm);
      }
    }
    if (cw >= 0) flush_walk(S, cw, acc, accm, lane);
  }
  PHASE_MARK(1);
  __syncthreads();
  PHASE_MARK(2);
  if (tid < nw) resolve_walk<SEG, true>(S, tid);
#ifndef FSCLG_SEGSTATS
  if (tid == 0) S.cnt[6] += (unsigned long long)S.n_ties;
#endif
  __syncthreads();
  PHASE_MARK(3);
#undef PHASE_MARK
}

// agent-scope atomics: performed at the memory side, coherent across the XCDs' L2s
__device__ __forceinline__ unsigned long long ag_add64(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ag_add32(unsigned int* p, unsigned int v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ag_or32(unsigned int* p, unsigned int v) {
  return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned int ag_xor32(unsigned int* p, unsigned int v) {
  return __hip_atomic_fetch_xor(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ag_xchg64(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Split cells: the members of a cell have each summed their segments of every walk into LDS;
// each writes its sums, parity words and ties into its own slots of the cell's exchange area
// for this instance, they meet at the cell's arrival counter (release / acquire at agent
// scope: the members may sit on different XCDs), and every member reads all slots and
// combines them identically, so that every member continues with the same values (resolve,
// argmax and bisection then run redundantly and agree).  Three memory round trips: the
// stores' completion, the arrival, the reads.  A member that waits longer than ~1 s (the
// others never started: not co-resident) flags the cell and goes on.
template <class SM>
__device__ __forceinline__ void combine_members(SM& S, const Params& P, int nw) {
  const int tid = threadIdx.x;
  const int inst = S.inst, me = S.member, G = P.split;
  XAcc* R = reinterpret_cast<XAcc*>(P.xacc + ((size_t)S.cell * 2 + (size_t)(inst & 1)) * sizeof(XAcc));
  // 1. this member's slots
  if (tid < nw) {
    R->P[me][tid] = S.P[tid];
    R->Q[me][tid] = S.Q[tid];
    R->wflag[me][tid] = (unsigned)S.wflag[tid];
    R->Pd[me][tid] = S.Pd[tid];
    R->Qd[me][tid] = S.Qd[tid];
#pragma unroll
    for (int j = 0; j < SEGWORDS; j++) R->segbits[me][tid][j] = S.segbits[tid][j];
  }
  {
    const int nt = S.n_ties;
    if (tid < min(nt, XTIES)) R->ties[me][tid] = S.ties[tid];
    if (tid == 0) R->nt[me] = (unsigned)nt;
  }
  // 2. arrive (release) and wait for every member (acquire)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned int* cnt = P.xcnt + S.cell;
    if (P.xdelay && inst == 0 && me == 0 && S.cell == 0) {  // tests: a member that is late by more than the wait
      const unsigned long long td = wall_clock64();
      while (wall_clock64() - td < P.xdelay) __builtin_amdgcn_s_sleep(127);
    }
    ag_add32(cnt, 1u);
    const unsigned int target = (unsigned)G * (unsigned)(inst + 1);
    const unsigned long long t0 = wall_clock64();
    unsigned int v;
    while (((v = ag_add32(cnt, 0u)) & ~XFAIL_BIT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > P.xwait) {  // a member never arrived: publish it for the whole cell
        S.xfail = PF_SPLIT_TIMEOUT;
        ag_or32(cnt, XFAIL_BIT);
        break;
      }
    }
    // Another member timed out (it went on with partial sums and may have overwritten this
    // instance's region), or more arrivals than members one instance ahead can make: either way
    // this cell's sums are not the reference's, and member 0 flags its point for the unsplit
    // re-run.  A member's flag precedes its later arrivals in the counter's order, so any
    // arrival a waiting member counted carries the flag of a timeout before it.
    if ((v & XFAIL_BIT) || (v & ~XFAIL_BIT) >= target + (unsigned)G) S.xfail = PF_SPLIT_TIMEOUT;
#ifdef FSCLG_PHASE_TIMING
    S.tph[4] += wall_clock64() - t0;
#endif
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 3. every member's slots, combined (all loads of this step in flight together)
  int tv = 0;
  bool th = false;
  {
    const int m = tid / XTIES, k = tid % XTIES;
    if (m < G) {
      const unsigned int ntm = R->nt[m];
      th = k < (int)min(ntm, (unsigned)XTIES);
      if (th) tv = R->ties[m][k];
    }
  }
  if (tid < nw) {
    unsigned long long pp = 0, qq = 0;
    unsigned int fl = 0, sb[SEGWORDS];
#pragma unroll
    for (int j = 0; j < SEGWORDS; j++) sb[j] = 0;
    for (int m = 0; m < G; m++) {
      pp += R->P[m][tid];
      qq += R->Q[m][tid];
      fl |= R->wflag[m][tid];
#pragma unroll
      for (int j = 0; j < SEGWORDS; j++) sb[j] ^= R->segbits[m][tid][j];
    }
    S.P[tid] = pp; S.Q[tid] = qq; S.wflag[tid] = (int)fl;
#pragma unroll
    for (int j = 0; j < SEGWORDS; j++) S.segbits[tid][j] = sb[j];
    if (fl) {
      double pd = 0.0, qd = 0.0;
      for (int m = 0; m < G; m++) {  // member order: the same sum on every member
        if (R->wflag[m][tid]) { pd += R->Pd[m][tid]; qd += R->Qd[m][tid]; }
      }
      S.Pd[tid] = pd; S.Qd[tid] = qd;
    }
  }
  if (tid < G) S.xnt[tid] = (int)R->nt[tid];
  __syncthreads();
  // 4. the ties, concatenated in member order (a member past XTIES: the overflow path)
  {
    const int m = tid / XTIES, k = tid % XTIES;
    int base = 0, tot = 0;
    bool over = false;
    for (int j = 0; j < G; j++) {
      const int n = S.xnt[j];
      if (j < m) base += min(n, XTIES);
      tot += n;
      over = over || n > XTIES;
    }
    if (th) S.ties[base + k] = tv;
    if (tid == 0) S.n_ties = over ? MAXTIES + 1 : tot;  // above MAXTIES marks the overflow as before
  }
  if (tid == 0) S.inst = inst + 1;
  __syncthreads();
}

template <bool LDS, bool SPLIT, class SM>
__device__ __forceinline__ void eval_walks(SM& S, const Params& P) {
  if constexpr (SM::HAS_BAND && LDS && !SPLIT) {
    if (P.band_th >= 0 && P.n_civ > 0) {  // band mode (FSCLG_BAND_TH=-1: the walk-window groups below)
      eval_walks_band<LDS>(S, P);
      return;
    }
  }
  constexpr int SEGN = SPLIT ? SEG_SPLIT : SEG;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = __builtin_amdgcn_readfirstlane(S.nwalk);
#ifdef FSCLG_PHASE_TIMING
  unsigned long long t0 = 0;
  if (tid == 0) t0 = wall_clock64();
#define PHASE_MARK(k) do { if (tid == 0) { const unsigned long long t1 = wall_clock64(); S.tph[k] += t1 - t0; t0 = t1; } } while (0)
#else
#define PHASE_MARK(k) do { } while (0)
#endif
  walk_bounds_par(S, P, tid, nw);
  if (tid < nw) {
    S.P[tid] = 0; S.Q[tid] = 0; S.Pd[tid] = 0.0; S.Qd[tid] = 0.0; S.wflag[tid] = 0; S.need_slow[tid] = 0;
    for (int j = 0; j < SEGWORDS; j++) S.segbits[tid][j] = 0;
  }
  if (tid == 0) S.n_ties = 0;
  __syncthreads();
  IEV(1, nw, 0);  // bounds done
  PHASE_MARK(0);  // FSCLG_PHASE_TIMING slots: 0 bounds + layout, 1 wave 0's segments, 2 the wait for
                  // the other waves, 3 the members' combine + resolve
  TRACE("  bounds done: nw=%d w0 len=%d nl=%d nr=%d\n", nw, S.w[0].len, S.w[0].nl, S.w[0].nr);
  // layout by wave 0, one lane per walk (nw <= 64), values in registers
  if (wave == 0) {
    const bool act = lane < nw;
    const int K = P.n_civ;
    int len = 0, wb = -1, nseg = 0;  // empty walks (wb = -1) sort last and open no group
    if (act) {
      Walk& W = S.w[lane];
      len = W.len ? 1 + W.nl + W.nr : 0;
      // the walk's window: the n_civ intervals below the one of its largest x (the site
      // count of a long walk grows like e^x up to there)
      if (LDS && K > 0 && len) {
        const int top = interval_of<LDS>(fmax(W.xl, W.xr), S, P);
        wb = min(max(top - K + 1, 0), P.n_iv - K);
      }
      const int near = S.pt[W.p].nearest, lo = near - W.nl, hi = near + W.nr;
      int nsl;
      if (!len) { nsl = 0; nseg = 0; }
      else { int nsr; seg_counts<SEGN>(lo, near, hi, nsl, nsr); nseg = nsl + nsr; }
      W.len = len; W.wb = wb; W.nsl = nsl; W.nseg = nseg;
    }
    // walks in descending window base, stable: each walk's rank and first segment
    int rank = 0, seg0 = 0;
    for (int j = 0; j < nw; j++) {
      const int wbj = __builtin_amdgcn_readlane(wb, j), nsj = __builtin_amdgcn_readlane(nseg, j);  // j uniform
      const bool before = wbj > wb || (wbj == wb && j < lane);
      rank += before ? 1 : 0;
      seg0 += before ? nsj : 0;
    }
    if (act) { S.w[lane].seg0 = seg0; S.word[rank] = lane; }
    // a group shares the window of its first walk and takes the following walks whose base
    // is at most 2 below it (they lose at most their two sparsest intervals)
    int ng = 0, gprev = 0;
    for (int k = 0; k < nw; k++) {
      const int l = __ffsll((unsigned long long)__ballot(act && rank == k)) - 1;
      const int wbk = __builtin_amdgcn_readlane(wb, l), lenk = __builtin_amdgcn_readlane(len, l),
                s0k = __builtin_amdgcn_readlane(seg0, l);
      if (lenk && (ng == 0 || wbk < gprev - FSCLG_GROUP_TOL)) {
        if (lane == 0) { S.gwb[ng] = wbk; S.gseg[ng] = s0k; S.gk[ng] = k; }
        ng++;
        gprev = wbk;
      }
    }
    int tot = nseg;
    long long terms = len;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { tot += __shfl_xor(tot, o, 64); terms += __shfl_xor(terms, o, 64); }
    if (lane == 0) {
      S.gseg[ng] = tot;
      S.gk[ng] = nw;
      S.ngrp = ng;
      S.seg_total = tot;
      S.cnt[0] += (unsigned long long)terms;
      S.cnt[2] += nw;
    }
  }
  __syncthreads();
  IEV(2, S.seg_total, S.ngrp);  // layout done
  PHASE_MARK(0);
  TRACE("  layout done: segs=%d\n", S.seg_total);
  // static round-robin of the equal-size segments over the waves; the loop
  // counter lives in an SGPR (a per-lane atomic-dispatch loop here was
  // miscompiled into a loop that never re-issued its atomic)
  {
    const int ngrp = __builtin_amdgcn_readfirstlane(S.ngrp);
    int k = 0, cw = -1, nsg_run = 0;
    double acc = 0.0, accm = 0.0;
    for (int gi = 0; gi < ngrp; gi++) {
     const int gwb = __builtin_amdgcn_readfirstlane(S.gwb[gi]);
     if (LDS && P.n_civ > 0 && gwb != __builtin_amdgcn_readfirstlane(S.ivc0)) {  // uniform over the workgroup
       __syncthreads();
       load_window(S, P, gwb);
       __syncthreads();
     }
     const int ge = __builtin_amdgcn_readfirstlane(S.gseg[gi + 1]);
     // split cells: the members deal the segments round-robin
     const int mstride = SPLIT ? NWAVE * P.split : NWAVE;
     const int g0 = SPLIT ? __builtin_amdgcn_readfirstlane(S.member) * NWAVE + wave : wave;
#if FSCLG_SITE_MAJOR
     // site-major: the group's ids run over the slices (j, part) = (0, left), (0, right), (1, left), ...;
     // slice (j, part) holds, in walk order, the walks whose part has more than j segments (lane l of
     // every wave holds the group's l-th walk and its part counts); id -> (walk, segment) by a ballot
     const int k0 = __builtin_amdgcn_readfirstlane(S.gk[gi]), nwg = __builtin_amdgcn_readfirstlane(S.gk[gi + 1]) - k0;
     int wl = 0, nsl_l = 0, nsr_l = 0;
     if (lane < nwg) { wl = S.word[k0 + lane]; nsl_l = S.w[wl].nsl; nsr_l = S.w[wl].nseg - nsl_l; }
#if FSCLG_FAR_FIRST
     // the slices from the farthest inwards: the phase ends on the dense near slices (every walk
     // reaches them), so the waves run out of work together
     int jmax = max(nsl_l, nsr_l) - 1;
#pragma unroll
     for (int o = 32; o > 0; o >>= 1) jmax = max(jmax, __shfl_xor(jmax, o, 64));
     jmax = __builtin_amdgcn_readfirstlane(jmax);
     int base = __builtin_amdgcn_readfirstlane(S.gseg[gi]), sj = jmax, spart = 0;
#else
     int base = __builtin_amdgcn_readfirstlane(S.gseg[gi]), sj = 0, spart = 0;
#endif
     unsigned long long M = __ballot(lane < nwg && (spart ? nsr_l : nsl_l) > sj);
     (void)k;
#endif
     for (int g = __builtin_amdgcn_readfirstlane(S.gseg[gi]) + g0; g < ge; g += mstride) {
#if FSCLG_SITE_MAJOR
#if FSCLG_FAR_FIRST
      while (g >= base + (int)__popcll(M) && sj >= 0) {  // g < ge: a later slice holds it
        base += (int)__popcll(M);
        if (spart == 0) spart = 1; else { spart = 0; sj--; }
#else
      while (g >= base + (int)__popcll(M) && sj < MAXSEG_W) {  // g < ge: a later slice holds it
        base += (int)__popcll(M);
        if (spart == 0) spart = 1; else { spart = 0; sj++; }
#endif
        M = __ballot(lane < nwg && (!FSCLG_FAR_FIRST || sj >= 0) && (spart ? nsr_l : nsl_l) > sj);
      }
      if (g >= base + (int)__popcll(M)) break;  // never: the slices hold exactly the group's segments
      const int rk = g - base;  // the rk-th walk of the slice
      const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(M >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)M, 0u));
      const int l = __ffsll(__ballot(((M >> lane) & 1ull) && below == rk)) - 1;
      const int w = __builtin_amdgcn_readlane(wl, l);
      const int sg = spart ? __builtin_amdgcn_readlane(nsl_l, l) + sj : __builtin_amdgcn_readlane(nsl_l, l) - 1 - sj;
#else
      while (k < nw - 1 && g >= S.w[S.word[k]].seg0 + S.w[S.word[k]].nseg) k++;  // walks own consecutive segment ranges
      const int w = S.word[k];
      const int sg = g - S.w[w].seg0;
#endif
      if (w != cw) {  // walk-major: the wave's segments of one walk are consecutive, one flush per walk
        if (cw >= 0) flush_walk(S, cw, acc, accm, lane);
        cw = w; acc = 0.0; accm = 0.0;
      }
#ifdef FSCLG_SEGSTATS
      if (lane == 0) atomicAdd(&S.cnt[6], 1ull);
#endif
      run_segment_idx<LDS, SEGN, SPLIT ? U_SPLIT : U_MAIN>(S, w, sg, sg + 1, P, lane, acc, accm);
      nsg_run++;
     }
    }
    if (cw >= 0) flush_walk(S, cw, acc, accm, lane);
    IEV(3, nsg_run, 0);  // wave 0's segment runs done
  }
  PHASE_MARK(1);
  __syncthreads();
  IEV(4, 0, 0);  // every wave's segments done
  PHASE_MARK(2);
  if constexpr (SPLIT) combine_members(S, P, nw);
  IEV(5, 0, 0);  // combined
  TRACE("  segments done: ties=%d\n", S.n_ties);
  if (tid < nw) resolve_walk<SEGN>(S, tid);
#ifndef FSCLG_SEGSTATS
  if (tid == 0) S.cnt[6] += (unsigned long long)S.n_ties;
#endif
  __syncthreads();
  IEV(6, 0, 0);  // resolved
  PHASE_MARK(3);
#undef PHASE_MARK
  TRACE("eval_walks: nw=%d segs=%d ties=%d\n", nw, S.seg_total, S.n_ties);
  (void)wave;
}

// sequential argmax with strict '>' (sm-search.c:279,287) over exact values,
// starting from a prior (the -DBL_MAX / LOG_AD_MAX initial state of
// sm-search.c:272, or the coarse winner in the refine phase).  Returns the
// winning walk, PRIOR if nothing beats the prior, or AMBIG after marking every
// inexact candidate that could still win for the sequential slow path.
constexpr int PRIOR = -1, AMBIG = -2;
template <class SM>
__device__ __forceinline__ int argmax_or_mark(SM& S, int first, int count, double prior_val) {
  int bi = PRIOR;
  double bv = prior_val;
  for (int c = first; c < first + count; c++)
    if (S.exact[c] && S.val[c] > bv) { bi = c; bv = S.val[c]; }
  // the best lower bound, inexact candidates included: a candidate whose upper bound is below
  // it cannot be the maximum (only the rest need their exact value)
  double lb = bv;
  for (int c = first; c < first + count; c++)
    if (!S.exact[c] && S.appr[c] - S.bnd[c] > lb) lb = S.appr[c] - S.bnd[c];
  int amb = 0;
  for (int c = first; c < first + count; c++)
    if (!S.exact[c] && !(S.appr[c] + S.bnd[c] < lb)) { S.need_slow[c] = 1; amb = 1; }
  return amb ? AMBIG : bi;
}

__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// argmax_or_mark by one wave, lane c holding candidate first + c (count <= 64): the sequential
// loop's winner is the first exact candidate holding the largest exact value above the prior
// (strict '>': a later equal value never replaces it; NaN never wins); the best lower bound and
// the marks as there.  Every lane returns the result.
template <class SM>
__device__ __forceinline__ int argmax_wave(SM& S, int first, int count, double prior_val, int lane) {
  const bool in = lane < count;
  const int c = first + (in ? lane : 0);
  const bool ex = in && S.exact[c] != 0;
  const double v = S.val[c], a = S.appr[c], b = S.bnd[c];
  const bool cand = ex && v > prior_val;
  const unsigned long long cm = __ballot(cand);
  int bi = PRIOR;
  double bv = prior_val;
  if (cm) {
    bv = wave_max_f64(cand ? v : -__builtin_inf());
    bi = first + __ffsll(__ballot(cand && v == bv)) - 1;
  }
  const bool inx = in && !ex;
  const double lb = fmax(bv, wave_max_f64(inx ? a - b : -__builtin_inf()));  // NaN bounds ignored, as '>' does
  const bool mark = inx && !(a + b < lb);
  if (mark) S.need_slow[c] = 1;
  return __ballot(mark) ? AMBIG : bi;
}

// search_maxalpha for the points in slots [p0, p0+np) (sm-search.c:269-300): the coarse phase (11
// alpha, strict '>' from -DBL_MAX), then the refine phase around the coarse winner (14-15 alpha,
// strict '>' from the coarse best).  Split cells (latency-bound: every phase is a chain of walk
// bounds, segments, the members' combine and the argmax) may evaluate the refine walks of a
// GUESSED coarse winner (Pt::sg) in the coarse phase: for a point whose real coarse winner is the
// guess, those walks are exactly the refine phase's walks (same alpha, same exact sums), so its
// refine argmax runs on them at once; only the points whose guess missed take a second phase.
// The candidates, their values and the order of the strict '>' comparisons are the reference's
// either way; a wrong guess costs only its walks.
template <bool LDS, bool SPLIT = false, class SM>
__device__ __forceinline__ void search_maxalpha_pts(SM& S, const Params& P, int p0, int np) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nc = P.n_coarse;
  const bool spec = SPLIT && P.spec_refine && np * (nc + MAXREF) <= SM::MAXW;  // uniform
  if (tid < np) set_binade(S.pt[p0 + tid]);
  IEV(0, np, S.pt[p0].sweep);  // an alpha search starts
  TRACE("maxalpha: p0=%d np=%d sweep=%d N=%g\n", p0, np, S.pt[p0].sweep, S.pt[p0].N);
  // ---- coarse phase
  if (tid < np * nc) {
    const int p = tid / nc, a = tid % nc;
    S.w[tid].p = p0 + p;
    S.w[tid].la = P.la_coarse[a];
    S.w[tid].dfail = P.dfail[a];
    S.w[tid].kd = a;
    S.w[tid].len = 0; S.w[tid].nl = S.w[tid].nr = 0;
  }
  if (tid == 0) { S.nwalk = np * nc; S.cnt[3] += np; S.hkey = 0; }
  // refine walks for point p's list ci[p] (lane p), after the first `base` walks: wave 0, lane
  // p * MAXREF + r for walk r; returns (first << 8) | count of point p's walks in lane p and sets
  // S.nwalk (cnt[p] = 0: none for that point)
  auto lay_refine = [&](int ci, int cnt, int base) {
    int off = 0, nw = base;
    for (int p = 0; p < np; p++) {  // np <= 2, uniform
      const int cp = __builtin_amdgcn_readlane(cnt, p);
      if (lane == p) off = nw;
      nw += cp;
    }
    if (lane == 0) S.nwalk = nw;
    const int p = lane / MAXREF, r = lane % MAXREF;
    const int pc = p < np ? p : 0;
    const int cip = __shfl(ci, pc, 64), cntp = __shfl(cnt, pc, 64), offp = __shfl(off, pc, 64);
    if (p < np && r < cntp) {
      Walk& V = S.w[offp + r];
      V.p = p0 + p;
      V.la = P.la_refine[cip * MAXREF + r];
      V.dfail = P.dfail[nc + cip * MAXREF + r];
      V.kd = nc + cip * MAXREF + r;
      V.len = 0; V.nl = V.nr = 0;
    }
    return (off << 8) | cnt;
  };
  if (spec && wave == 0) {  // the guessed winners' refine walks, after the coarse walks
    int g = 0, cnt = 0;
    if (lane < np) { g = min(max(S.pt[p0 + lane].sg, 0), nc); cnt = P.n_refine[g]; }
    const int pad = lay_refine(g, cnt, np * nc);
    if (lane < np) { S.pt[p0 + lane].sg = g; S.pt[p0 + lane].spad = pad; }
  }
  __syncthreads();
  // argmax per point of `mask` over its coarse (refine = false) or refine walks (first, count in
  // Pt::pad), with slow-path settling; S.best[p] = the winning walk or PRIOR
  auto settle = [&](unsigned mask, bool refine) {
    for (int round = 0; round < 2; round++) {
      if (wave == 0) {
        int slow = 0;
        for (int p = 0; p < np; p++) {
          if (!((mask >> p) & 1u)) continue;  // uniform
          const Pt& pt = S.pt[p0 + p];
          int first, count;
          double pv;
          if (!refine) { first = p * nc; count = nc; pv = -1.7976931348623157e308; }
          else { first = pt.pad >> 8; count = pt.pad & 0xFF; pv = pt.sm; }
          const int r = argmax_wave(S, first, count, pv, lane);
          if (r == AMBIG) slow = 1;
          if (lane == 0) S.best[p] = r;
        }
        if (lane == 0) S.n_slow = slow;
      }
      __syncthreads();
      if (S.n_slow == 0) break;
      // settle marked walks exactly: one wave per walk
      const int nwk = __builtin_amdgcn_readfirstlane(S.nwalk);
      for (int w = wave; w < nwk; w += NWAVE) {
        if (__builtin_amdgcn_readfirstlane(S.need_slow[w])) {
          const double v = walk_sequential<LDS>(S, S.w[w], S.pt[S.w[w].p], P, lane);
          if (lane == 0) { S.val[w] = v; S.exact[w] = 1; S.need_slow[w] = 0; atomicAdd(&S.cnt[5], 1ull); }
        }
      }
      __syncthreads();
    }
  };
  // the refine argmax's result for the points of `mask` (sm-search.c:298 for every point)
  auto finish = [&](unsigned mask) {
    if (tid < np) {
      Pt& pt = S.pt[p0 + tid];
      const int bi = S.best[tid];
      if (((mask >> tid) & 1u) && bi != PRIOR) { pt.la = S.w[bi].la; pt.sm = S.val[bi]; }
      pt.clr = 2.0 * (pt.sm - pt.N);
    }
    __syncthreads();
  };
  const unsigned all = (1u << np) - 1u;
  eval_walks<LDS, SPLIT>(S, P);
  settle(all, false);
  // coarse winners (or the untouched initial state); the points whose guess held
  if (wave == 0) {
    bool hit = false;
    if (lane < np) {
      const int bi = S.best[lane];
      Pt& pt = S.pt[p0 + lane];
      int ci;
      if (bi == PRIOR) { pt.la = LOG_AD_MAX; pt.sm = -1.7976931348623157e308; ci = nc; }
      else { pt.la = S.w[bi].la; pt.sm = S.val[bi]; ci = bi - lane * nc; }
      pt.ci = ci;
      hit = spec && ci == pt.sg && P.spec_refine != 2;  // (FSCLG_SPEC_REFINE=2, tests: every guess taken as missed)
      if (hit) pt.pad = pt.spad;
    }
    const unsigned hm = (unsigned)__ballot(hit) & all;
    if (lane == 0) { S.hkey = 1 + S.pt[p0].ci; S.hitmask = (int)hm; }
  }
  __syncthreads();
  const unsigned hm = (unsigned)__builtin_amdgcn_readfirstlane(S.hitmask);
  if (hm) {  // refine argmax of the points whose speculative walks are the right ones
    settle(hm, true);
    finish(hm);
  }
  const unsigned miss = all & ~hm;
  if (miss) {  // ---- refine phase for the rest
    if (wave == 0) {
      int ci = 0, cnt = 0;
      if (lane < np && ((miss >> lane) & 1u)) { ci = S.pt[p0 + lane].ci; cnt = P.n_refine[ci]; }
      const int pad = lay_refine(ci, cnt, 0);
      if (lane < np && ((miss >> lane) & 1u)) S.pt[p0 + lane].pad = pad;
    }
    __syncthreads();
    eval_walks<LDS, SPLIT>(S, P);
    settle(miss, true);
    finish(miss);
  }
}

__device__ __forceinline__ void read_point(Pt& pt, const fsclg_point_t& in) {
  pt.chr = in.chr; pt.nearest = in.nearest_snp; pt.sweep = in.sweep_pos; pt.n_snps = in.n_snps;
  pt.wstart = in.window_start; pt.wend = in.window_end; pt.flags = in.flags;
  pt.la = in.lalpha; pt.N = in.null_logl; pt.sm = in.sm_logl; pt.clr = in.clr;
  set_binade(pt);
}

__device__ __forceinline__ void write_point(fsclg_point_t& o, const Pt& pt) {
  o.chr = pt.chr; o.nearest_snp = pt.nearest; o.sweep_pos = pt.sweep; o.n_snps = pt.n_snps;
  o.window_start = pt.wstart; o.window_end = pt.wend; o.flags = pt.flags; o.cost = 0;
  o.lalpha = pt.la; o.null_logl = pt.N; o.sm_logl = pt.sm; o.clr = pt.clr;
}

template <bool LDS, bool SPLIT, class SM>
__device__ __forceinline__ void maxpos_body(SM& S, const Params& P) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // cells arrive in the host's longest-first order (XCD-aware: blocks b and b + 8 share an
  // XCD); the hardware dispatches blocks in order (round-robin over the XCDs), so the long
  // cells start first and spread over the XCDs.  Split cells: the members of cell c are blocks
  // (c / 8) * 8G + 8m + c % 8, m < G -- one XCD's L2 holds the cell's sites
  const int G = SPLIT ? P.split : 1, b = (int)blockIdx.x;
  const int cell = G > 1 ? (b / (8 * G)) * 8 + (b & 7) : b;
  const int member = G > 1 ? (b >> 3) % G : 0;
  if (cell >= P.n_cells) return;
  if (P.mode == 0 && P.cells[cell].chr < 0) {  // idle block of the host's XCD placement
    if (P.ctrace && tid < 8) P.ctrace[8 * cell + tid] = 0;
    return;
  }
  if (tid < 8) S.cnt[tid] = 0;
  if (tid < 5) S.tph[tid] = 0;
  if (tid == 0) { S.cell = cell; S.member = member; S.inst = 0; S.xfail = 0; S.iev = 0; }
  if (P.ctrace && tid == 0 && member == 0) { P.ctrace[8 * cell] = wall_clock64(); P.ctrace[8 * cell + 2] = __smid(); }
  if constexpr (LDS) {
    double* thr = reinterpret_cast<double*>(fsclg_dyn + P.off_thr);
    double* nul = reinterpret_cast<double*>(fsclg_dyn + P.off_nul);
    for (int j = tid; j <= P.n_iv; j += WG) thr[j] = P.thr[j];
    for (int j = tid; j <= P.n_rows; j += WG) nul[j] = P.nullrow[j];  // + sentinel
    load_window(S, P, P.ivc0);
    double* lt2 = reinterpret_cast<double*>(fsclg_dyn + P.off_lt);
    for (int j = 256 + tid; j < P.lt_hi; j += WG) lt2[j] = P.logt3[2 * 0x10000 + j];
#if FSCLG_LOG_CALC
    if (lx_kernel<SM>() && P.lx_on) {
      double* lx = reinterpret_cast<double*>(fsclg_dyn + P.off_lx);
      for (int j = tid; j < LX_BYTES / 8; j += WG) lx[j] = P.lx[j];
    }
#endif
  } else if (tid == 0) S.ivc0 = 0;
  __syncthreads();
  if (P.mode == 1) {
    if (tid == 0) {
      const fsclg_point_t& in = P.out[cell];
      Pt& pt = S.pt[0];
      pt.chr = in.chr; pt.nearest = in.nearest_snp; pt.sweep = in.sweep_pos; pt.wstart = in.window_start;
      pt.wend = in.window_end; pt.n_snps = in.n_snps; pt.flags = 0; pt.N = in.null_logl;
    }
    __syncthreads();
    if (tid == 0) { S.cnt[1] += (unsigned long long)S.pt[0].n_snps; S.pt[0].sg = P.ci_guess; }
    __syncthreads();
    search_maxalpha_pts<LDS, SPLIT>(S, P, 0, 1);  // split: the point's walks dealt over the members
    if (tid == 0 && member == 0) {
      S.pt[0].flags |= S.xfail;
      write_point(P.out[cell], S.pt[0]);
    }
  } else if (P.mode == 2) {
    // distinct cell endpoints, two per block: scan-chromosome.c:130-134 for each
    const int e0 = 2 * cell, np = min(2, P.n_ep - e0);
    if (wave < np) init_point_wave(S.pt[wave], P.epos[e0 + wave].x, P.epos[e0 + wave].y, P, lane);
    __syncthreads();
    if (tid == 0) for (int k = 0; k < np; k++) S.cnt[1] += (unsigned long long)S.pt[k].n_snps;
    search_maxalpha_pts<LDS>(S, P, 0, np);
    if (tid < np) write_point(P.ept[e0 + tid], S.pt[tid]);
  } else {
    const fsclg_cell_t c = P.cells[cell];
    if (P.cell_ep) {  // endpoints evaluated by a mode-2 launch (shared with the neighbouring cells)
      if (tid < 2) { read_point(S.pt[tid], P.ept[tid == 0 ? P.cell_ep[cell].x : P.cell_ep[cell].y]); S.pt[tid].ci = P.ci_guess; }
      __syncthreads();
    } else {
      if (wave < 2) init_point_wave(S.pt[wave], c.chr, wave == 0 ? c.start_pos : c.end_pos, P, lane);
      __syncthreads();
      if (tid == 0) { S.cnt[1] += (unsigned long long)(S.pt[0].n_snps + S.pt[1].n_snps); S.pt[0].sg = S.pt[1].sg = P.ci_guess; }
      __syncthreads();
      search_maxalpha_pts<LDS, SPLIT>(S, P, 0, 2);  // start and end points share the two phases
    }
    // the bisection (scan-chromosome.c:103-139), two levels per alpha search: a level goes
    // left iff (s + m) >= (e + m) (compared exactly as written, :116).  IEEE addition is
    // monotone, so s >= e makes that true whatever m is, and otherwise it is false unless the
    // two sums round together (or m is NaN).  The next level's midpoint -- the middle of the
    // half that s >= e predicts -- is evaluated beside m; when the level's real decision
    // agrees (nearly always) that level is taken from it at once, otherwise it is dropped and
    // the next round evaluates the other half's midpoint.  The points evaluated on the path
    // and every comparison are the reference's; only the number of dependent searches halves.
    int iter = 0;
    for (;;) {
      const int sp = S.pt[0].sweep, ep = S.pt[1].sweep;
      if (ep - sp <= P.bp_resl) break;
      if (++iter > 64) { if (tid == 0) S.pt[0].flags |= PF_NOCONV; break; }
      // (FSCLG_LOOKAHEAD=2, tests: predict the other half, so every look-ahead point is dropped)
      const bool pleft = (S.pt[0].clr >= S.pt[1].clr) != (P.lookahead == 2);
      if (wave == 0) {
        init_point_wave(S.pt[2], c.chr, (sp + ep) / 2, P, lane);
        if (lane == 0) S.cnt[1] += (unsigned long long)S.pt[2].n_snps;
      }
      __syncthreads();
      // the predicted half ends at the midpoint's own position (init_scan_result may move a
      // point that sits on a SNP, scan-chromosome.c:67-71)
      const int m1 = S.pt[2].sweep;
      const int cs = pleft ? sp : m1, ce = pleft ? m1 : ep;
      const bool two = P.lookahead && ce - cs > P.bp_resl;
      if (two) {
        if (wave == 0) {
          init_point_wave(S.pt[3], c.chr, (cs + ce) / 2, P, lane);
          if (lane == 0) S.cnt[1] += (unsigned long long)S.pt[3].n_snps;
        }
        __syncthreads();
      }
      // split cells' speculative refine walks: the better end's coarse winner (the bisection
      // heads towards it, and a point's winner changes slowly along the chromosome)
      if (tid == 0) S.pt[2].sg = S.pt[3].sg = S.pt[0].clr >= S.pt[1].clr ? S.pt[0].ci : S.pt[1].ci;
      __syncthreads();
      search_maxalpha_pts<LDS, SPLIT>(S, P, 2, two ? 2 : 1);
      // every thread takes the same decisions from the same shared values (uniform control)
      const bool left = (S.pt[0].clr + S.pt[2].clr) >= (S.pt[1].clr + S.pt[2].clr);
      const bool lvl2 = two && left == pleft;  // the next level, its midpoint already evaluated
      if (lvl2) ++iter;
      __syncthreads();
      if (tid == 0) {
        if (left) S.pt[1] = S.pt[2];
        else S.pt[0] = S.pt[2];
        if (lvl2) {
          if (iter > 64) S.pt[0].flags |= PF_NOCONV;
          if ((S.pt[0].clr + S.pt[3].clr) >= (S.pt[1].clr + S.pt[3].clr)) S.pt[1] = S.pt[3];
          else S.pt[0] = S.pt[3];
        }
      }
      __syncthreads();
    }
    if (tid == 0 && member == 0) {  // one store of the result (P.out may be host memory: no read-modify-write)
      const Pt& r = S.pt[0].clr > S.pt[1].clr ? S.pt[0] : S.pt[1];
      fsclg_point_t o;
      write_point(o, r);
      o.flags |= S.pt[0].flags | S.pt[1].flags | S.xfail;
      o.cost = (uint32_t)min(S.cnt[0] >> 10, 0xFFFFFFFFull);
      P.out[cell] = o;
      S.cnt[7] += 1;
    }
  }
  __syncthreads();
  if (member != 0) return;  // split cells: member 0 reports (the others counted the same walks)
  if (tid < 8 && S.cnt[tid]) atomicAdd(&P.stats[tid], S.cnt[tid]);
  if (P.ctrace && tid == 0) {
    P.ctrace[8 * cell + 1] = wall_clock64(); P.ctrace[8 * cell + 3] = S.cnt[0];
    for (int k = 0; k < 4; k++) P.ctrace[8 * cell + 4 + k] = S.tph[k];
#ifdef FSCLG_PHASE_TIMING
    P.ctrace[8 * cell + 2] = S.tph[4] | ((unsigned long long)S.inst << 48);  // (the CU id's slot; + the phases)
#endif
  }
}

// waves per SIMD to budget registers for (caps VGPRs at 512 / waves): the throughput kernel
// runs two workgroups per CU (6 waves per SIMD); a split launch (few cells, latency) keeps
// its workgroups far apart and may spend more registers per wave on wider trips
#ifndef FSCLG_WPE_SPLIT
#define FSCLG_WPE_SPLIT 6
#endif
template <bool LDS, bool BAND = false>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(FSCLG_WPE, FSCLG_WPE)))
search_maxpos_kernel(Params P) {
  __shared__ SmemT<MAXWALK, BAND> S;
  maxpos_body<LDS, false>(S, P);
}

template <bool LDS>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(FSCLG_WPE_SPLIT, FSCLG_WPE_SPLIT)))
search_maxpos_split_kernel(Params P) {
  __shared__ SmemSplit S;
  maxpos_body<LDS, true>(S, P);
}

// ------------------------------------------------------------ window null sums
// init_scan_result's window sum (scan-chromosome.c:92-94) for every window start of the
// chromosomes longer than the window: acc = 0.0; acc += null_logl[i] for i = ws..ws+W-1,
// in that order, per window.  A thread carries WN_PER neighbouring windows (each element
// read once from LDS feeds all of them, each accumulator in its own ascending order); the
// block stages the elements its 1024 windows span through an LDS tile.
constexpr int WN_WG = 256, WN_PER = 4, WN_TILE = 4096;

// A block's staging of a tile is one round of independent row loads (all of a full tile's rows
// before any null value), and its sums read the tile eight elements at a time before adding
// them: each window's chain of adds then runs at the FP64 add latency, not one LDS round trip
// per element (measured: 20 ms per C5 x 4 launch before, one read and four adds per element).
template <int WPER>
__global__ void __launch_bounds__(WN_WG)
window_null_kernel(const uint2* __restrict__ pr, const double* __restrict__ nullrow, const int2* __restrict__ tasks,
                   int W, double* __restrict__ out) {
  __shared__ double tile[WN_TILE];
  // the search kernels' waves share these SIMDs and wait on memory most of their cycles; a
  // trial's cells wait for these sums, so their waves issue first
  __builtin_amdgcn_s_setprio(2);
  const int2 t = tasks[blockIdx.x];  // windows [t.x, t.x + t.y)
  const int k = threadIdx.x;
  const int base = t.x + WPER * k;
  const int nwin = min(max(t.y - WPER * k, 0), WPER);
  const int end = t.x + t.y - 1 + W;  // one past the last element a window of the block uses
  double a[WPER];
#pragma unroll
  for (int m = 0; m < WPER; m++) a[m] = 0.0;
  for (int T0 = t.x; T0 < end; T0 += WN_TILE) {
    const int T1 = min(T0 + WN_TILE, end);
    __syncthreads();
    if (T1 - T0 == WN_TILE) {
      uint32_t rr[WN_TILE / WN_WG];
#pragma unroll
      for (int q = 0; q < WN_TILE / WN_WG; q++) rr[q] = pr[phys((uint32_t)(T0 + k + q * WN_WG))].y;
#pragma unroll
      for (int q = 0; q < WN_TILE / WN_WG; q++) tile[k + q * WN_WG] = nullrow[rr[q]];
    } else {
      for (int j = T0 + k; j < T1; j += WN_WG) tile[j - T0] = nullrow[pr[phys((uint32_t)j)].y];
    }
    __syncthreads();
    if (nwin == 0) continue;
    const int lo = max(T0, base), hi = min(T1, base + nwin - 1 + W);
    // window m takes elements base + m .. base + m + W - 1
    auto edge = [&](int j0, int j1) {
      for (int j = j0; j < j1; j++) {
        const double v = tile[j - T0];
        const int off = j - base;
#pragma unroll
        for (int m = 0; m < WPER; m++)
          if (m < nwin && off >= m && off < W + m) a[m] += v;
      }
    };
    if (nwin < WPER) { edge(lo, hi); continue; }
    const int m0 = min(max(lo, base + WPER - 1), hi), m1 = max(min(hi, base + W), m0);
    edge(lo, m0);
    int j = m0;
    for (; j + 8 <= m1; j += 8) {  // every window of the thread takes these, each in order
      double v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = tile[j - T0 + q];
#pragma unroll
      for (int q = 0; q < 8; q++)
#pragma unroll
        for (int m = 0; m < WPER; m++) a[m] += v[q];
    }
    for (; j < m1; j++) {
      const double v = tile[j - T0];
#pragma unroll
      for (int m = 0; m < WPER; m++) a[m] += v;
    }
    edge(m1, hi);
  }
#pragma unroll
  for (int m = 0; m < WPER; m++)
    if (m < nwin) out[base + m] = a[m];
}

// ------------------------------------------------ window null sums by exact chunks
// The same sums (acc = 0.0; acc += null_logl[i], i = ws..ws+W-1, sequentially) with most of the
// 2 er + 1 dependent adds replaced by one step per aligned 64-site chunk.
// While the running sum S stays in one binade, |S| in [2^e, 2^(e+1)), every sequential add rounds
// to the grid u = 2^(e-52): with S = m u (m an integer, |m| in [2^52, 2^53)) and q = v / u
// (exact: a power-of-two scaling), fl(S + v) = (m + rint(q)) u, except at a tie (q = F + 1/2),
// which rounds to the even neighbour: m + F + ((m + F) & 1).  After a tie m is even, so a chunk's
// total increment depends on S only through the parity of m on entry: two integers per (chunk,
// binade), chunk_table_kernel.  Null values are log-probabilities (<= 0), so the partial sums are
// monotone and a chunk stays in the binade iff its end does; a chunk that crosses into the next
// binade, one holding a positive or non-finite value (NaN in the table), the windows' ends and
// the first sites (until |S| >= 2^emin, where a binade spans at least a chunk) are added site by
// site in order.  Same result as the sequential chain, bit for bit, for every window.
constexpr int WC = 64;   // chunk length, aligned to the site index
constexpr int WCG = 16;  // chunks per wave-uniform group (their table entries: one scalar load run)

// binade e = emin + k, chunk c: tab[k * nstride + c] = (d0, d1 - d0), d0 / d1 the increment of the
// chunk's 64 sequential adds for an even / odd m on entry, exact doubles (|increment| < 2^52 by the
// choice of emin), so that the increment is fma(parity, d1 - d0, d0), exactly; NaN when the chunk holds a value that is positive, not finite, or lies past the last
// site.  Binade-major, so that a group of consecutive chunks at one binade is one contiguous run;
// nstride = chunks + WCG (the padding entries are NaN).
#ifndef FSCLG_CT_BG
#define FSCLG_CT_BG 8
#endif
constexpr int CT_BG = FSCLG_CT_BG;  // binades per thread: each chunk's 64 null values are read once per CT_BG binades
__global__ void __launch_bounds__(256) chunk_table_kernel(const uint2* __restrict__ pr,
                                                          const double* __restrict__ nullrow, int n_snps, int emin,
                                                          int ne, int nstride, double2* __restrict__ tab) {
  const int ng = (ne + CT_BG - 1) / CT_BG;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= nstride * ng) return;
  const int grp = t / nstride, c = t - grp * nstride, k0 = grp * CT_BG;
  const double nan = __longlong_as_double(0x7FF8000000000000ll);
  if ((c + 1) * WC > n_snps) {
    for (int k = k0; k < ne && k < k0 + CT_BG; k++) tab[(size_t)k * nstride + c] = make_double2(nan, nan);
    return;
  }
  // per binade e = emin + k: the running integer's increments from entry parity 0 and 1 (exact
  // below 2^52: 64 values of magnitude < 2^e / 64 each, scaled by 2^(52 - e))
  double d0[CT_BG], d1[CT_BG];
  int p0[CT_BG], p1[CT_BG];
#pragma unroll
  for (int b = 0; b < CT_BG; b++) { d0[b] = 0.0; d1[b] = 0.0; p0[b] = 0; p1[b] = 1; }
  bool ok = true;
  for (int j = 0; j < WC; j++) {
    const double v = nullrow[pr[phys((uint32_t)(c * WC + j))].y];
    if (!(v <= 0.0) || v == -__builtin_inf()) { ok = false; break; }  // positive, NaN or -inf
#pragma unroll
    for (int b = 0; b < CT_BG; b++) {
      const int e = emin + k0 + b;  // e <= 52 for the entries written; the others are computed and dropped
      const double sc = __longlong_as_double((long long)(1023 + 52 - (e < 52 ? e : 52)) << 52);  // 2^(52 - e)
      const double q = v * sc;
      const double F = floor(q);
      if (q - F == 0.5) {
        const long long Fi = (long long)F;
        d0[b] += (double)(Fi + ((p0[b] + Fi) & 1)); p0[b] = 0;
        d1[b] += (double)(Fi + ((p1[b] + Fi) & 1)); p1[b] = 0;
      } else {
        const double R = rint(q);
        const int Rp = (int)((long long)R & 1);
        d0[b] += R; p0[b] = (p0[b] + Rp) & 1;
        d1[b] += R; p1[b] = (p1[b] + Rp) & 1;
      }
    }
  }
#pragma unroll
  for (int b = 0; b < CT_BG; b++)
    if (k0 + b < ne)
      tab[(size_t)(k0 + b) * nstride + c] = ok ? make_double2(d0[b], d1[b] - d0[b]) : make_double2(nan, nan);
}

// Block maps.  Within one binade a chunk's increment depends on the running
// integer m only through its parity (chunk_table_kernel: (d0, d1 - d0)), so the map of a run of
// chunks is again m -> m + D[m & 1], and maps compose: the run [a, c) after [a, b) gives
// D[p] = D1[p] + D2[(p + D1[p]) & 1].  chunk_tree_kernel composes the chunk table over aligned
// blocks of 2^L chunks, L = 1 .. lmax, so that a window's interior takes O(log) steps instead of
// one per chunk.  The partial sums are monotone (every null value <= 0), so a block keeps m in
// its binade iff its end does, the same test as for one chunk.  Exactness: a block that can keep
// any m in (-2^53, -2^52] inside has |D| < 2^53, an exact double; a larger |D| may round, but then
// it is at least 2^53 in magnitude and fails the test anyway.  NaN (a positive, NaN or -inf null
// value, or the padding past the last site) propagates through the composition.
constexpr int CT_LMAX = 12;
struct CTree {
  const double2* p;              // level L >= 1, binade k, block b at p[off[L] + k * nb[L] + b]
  int lmax;                      // 0: no blocks (one step per chunk, in groups of WCG)
  int off[CT_LMAX + 1], nb[CT_LMAX + 1];
};

__device__ __forceinline__ double2 compose_maps(double2 f1, double2 f2) {
  const double a0 = f1.x, a1 = f1.x + f1.y, b0 = f2.x, b1 = f2.x + f2.y;
  const double D0 = a0 + ((((long long)a0) & 1ll) ? b1 : b0);       // entry parity 0
  const double D1 = a1 + ((((long long)a1 + 1ll) & 1ll) ? b1 : b0);  // entry parity 1
  return make_double2(D0, D1 - D0);
}

// The same table with the chunks' null values staged through LDS: a workgroup loads the 4096
// values of 64 consecutive chunks with coalesced reads (one site per thread per pass) and stores them
// transposed (tile[j][chunk], a row padded to 65 doubles), so that its four waves -- lane = chunk,
// wave = a group of CT_BGL binades -- read their chunk's j-th value conflict-free.  chunk_table_kernel
// reads each chunk's sites with one lane per chunk, 64 lanes 1 KB apart, per load.  A wave's 64
// chunks are one aligned block of level 6, so it also composes the block maps of levels 1 .. nlev
// (nlev <= CT_SPAN) across its lanes, as chunk_tree_kernel does, before anything is written back.
constexpr int CT_BGL = 3;  // binades per lane per pass (4 waves x 3: C5's 12 binades in one pass)
__global__ void __launch_bounds__(256) chunk_table_lds_kernel(const uint2* __restrict__ pr,
                                                              const double* __restrict__ nullrow, int n_snps,
                                                              int emin, int ne, int nstride,
                                                              double2* __restrict__ tab, CTree T,
                                                              double2* __restrict__ tree, int nlev) {
  __shared__ double tile[WC][65];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c0 = blockIdx.x * 64;
  const double nan = __longlong_as_double(0x7FF8000000000000ll);
#pragma unroll 4
  for (int q = 0; q < WC * 64 / 256; q++) {
    const int k = q * 256 + t, sidx = c0 * WC + k;  // k: the block's k-th site, chunk k >> 6, index k & 63
    tile[k & 63][k >> 6] = sidx < n_snps ? nullrow[pr[phys((uint32_t)sidx)].y] : nan;
  }
  __syncthreads();
  const int c = c0 + lane;  // chunks past nstride: NaN, composed but never written
  const bool whole = (c + 1) * WC <= n_snps;
  for (int k0 = wave * CT_BGL; k0 < ne; k0 += 4 * CT_BGL) {
    double d0[CT_BGL], d1[CT_BGL];
    int p0[CT_BGL], p1[CT_BGL];
#pragma unroll
    for (int b = 0; b < CT_BGL; b++) { d0[b] = 0.0; d1[b] = 0.0; p0[b] = 0; p1[b] = 1; }
    bool ok = whole;
    for (int j = 0; j < WC && ok; j++) {
      const double v = tile[j][lane];
      if (!(v <= 0.0) || v == -__builtin_inf()) { ok = false; break; }  // positive, NaN or -inf
#pragma unroll
      for (int b = 0; b < CT_BGL; b++) {
        const int e = emin + k0 + b;  // e <= 52 for the entries written; the others are computed and dropped
        const double sc = __longlong_as_double((long long)(1023 + 52 - (e < 52 ? e : 52)) << 52);  // 2^(52 - e)
        const double q = v * sc;
        const double F = floor(q);
        if (q - F == 0.5) {
          const long long Fi = (long long)F;
          d0[b] += (double)(Fi + ((p0[b] + Fi) & 1)); p0[b] = 0;
          d1[b] += (double)(Fi + ((p1[b] + Fi) & 1)); p1[b] = 0;
        } else {
          const double R = rint(q);
          const int Rp = (int)((long long)R & 1);
          d0[b] += R; p0[b] = (p0[b] + Rp) & 1;
          d1[b] += R; p1[b] = (p1[b] + Rp) & 1;
        }
      }
    }
#pragma unroll
    for (int b = 0; b < CT_BGL; b++) {
      const int k = k0 + b;
      if (k >= ne) continue;  // uniform
      double2 v = ok ? make_double2(d0[b], d1[b] - d0[b]) : make_double2(nan, nan);
      if (c < nstride) tab[(size_t)k * nstride + c] = v;
      for (int l = 0; l < nlev; l++) {
        const int st = 1 << l, L = l + 1;
        const double2 r = make_double2(__shfl_down(v.x, st, 64), __shfl_down(v.y, st, 64));
        if ((lane & (2 * st - 1)) == 0) {
          v = compose_maps(v, r);
          const int bb = c >> L;
          if (bb < T.nb[L]) tree[T.off[L] + (size_t)k * T.nb[L] + bb] = v;
        }
      }
    }
  }
}

// levels L0 .. L0 + nlev - 1 of the block maps, nlev <= CT_SPAN: each wave takes 64 consecutive
// entries of level L0 - 1 (level 0: the chunk table) of one binade, one per lane, and composes them
// level by level across its lanes (lane i holds the block starting at entry i once i is a multiple
// of its size), writing each level's blocks that exist (block b of level L covers entries 2b,
// 2b + 1 of level L - 1; level L has nb[L] = chunks >> L blocks).  No LDS, so the kernel runs
// beside search workgroups that hold all of it; two launches cover 12 levels (ensure_ctab).
constexpr int CT_SPAN = 6;
__global__ void __launch_bounds__(256) chunk_tree_kernel(const double2* __restrict__ ctab, int nstride, CTree T,
                                                         double2* __restrict__ out, int L0, int nlev, int ngrp) {
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x / ngrp, g = (blockIdx.x - k * ngrp) * 4 + (threadIdx.x >> 6);  // wave g of binade k
  const int nprev = L0 == 1 ? nstride : T.nb[L0 - 1];
  const double2* prev = L0 == 1 ? ctab + (size_t)k * nstride : out + T.off[L0 - 1] + (size_t)k * T.nb[L0 - 1];
  const long long i0 = (long long)g * 64 + lane;
  double2 v = i0 < nprev ? prev[i0] : make_double2(__longlong_as_double(0x7FF8000000000000ll), 0.0);
  for (int l = 0; l < nlev; l++) {
    const int st = 1 << l, L = L0 + l;
    const double2 r = make_double2(__shfl_down(v.x, st, 64), __shfl_down(v.y, st, 64));
    if ((lane & (2 * st - 1)) == 0) {
      v = compose_maps(v, r);
      const long long b = ((long long)g * 64 + lane) >> (l + 1);
      if (b < T.nb[L]) out[T.off[L] + (size_t)k * T.nb[L] + b] = v;
    }
  }
}

// A wave sums the windows of 64 consecutive starts (one per lane; 256 per block, tasks: [start,
// count]), walking the absolute chunks in order, every lane at the same chunk:
//  * interior groups: while every lane is at a whole chunk of its window, at least 2^emin in
//    magnitude and in one binade e, WCG chunks' entries for e are read by the whole wave at once
//    (uniform address: scalar loads), and each chunk is one add per lane on the integer m; a chunk
//    that some lane would leave the binade with (or a NaN entry) ends the group and goes to
//  * the general step: each lane takes its chunk from the table when it can (its own entry), or
//    adds the chunk's sites of its window in order, the chunk's null values loaded by the wave
//    (one site per lane) and broadcast lane by lane.
// The windows' ends, the first sites (until |S| >= 2^emin) and the binade crossings take the
// general step; lanes' sums differ by their first few sites only, so they cross together.
__global__ void __launch_bounds__(WN_WG)
window_chunk_kernel(const uint2* __restrict__ pr, const double* __restrict__ nullrow,
                    const int2* __restrict__ tasks, int W, int emin, int ne, int nstride,
                    const double2* __restrict__ tab, double* __restrict__ out, CTree T, int wdesc) {
  __builtin_amdgcn_s_setprio(2);  // beside the search kernels' waves, which wait on memory
  const int2 t = tasks[blockIdx.x];
  const int lane = threadIdx.x & 63;
  const int w0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));  // the wave's first window in the block
  if (w0 >= t.y) return;
  const int nv = min(64, t.y - w0);
  const bool valid = lane < nv;
  const int ws0 = t.x + w0, wsL = ws0 + nv - 1;
  const int ws = ws0 + min(lane, nv - 1), end = ws + W;  // invalid lanes shadow the last valid one
  double s = 0.0;
  const int cend = ((wsL + W - 1) >> 6) + 1;
  const int fast_lo = (wsL + WC - 1) >> 6;  // chunks at or past every lane's start
  const int fast_hi = (ws0 + W) >> 6;       // chunks ending at or before every lane's end
  const double TWO53 = 9007199254740992.0;
  int c = ws0 >> 6;
  while (c < cend) {
    if (c >= fast_lo && c < fast_hi) {  // uniform (c stays uniform: every branch that moves it is)
      const int e = (int)((__double_as_longlong(s) >> 52) & 0x7FF) - 1023;
      const int eu = __builtin_amdgcn_readfirstlane(e);
      if (eu >= emin && eu < emin + ne && __builtin_amdgcn_ballot_w64(!(s < 0.0) || e != eu) == 0ull &&
          T.lmax > 0) {
        // block steps: the largest aligned block at c that ends by fast_hi; on a binade crossing
        // (or a NaN block) the same c with half the block, down to one chunk, then the general step
        typedef const __attribute__((address_space(4))) double cdouble;
        const double sc = __longlong_as_double((long long)(1023 + 52 - eu) << 52);   // 2^(52 - e)
        const double isc = __longlong_as_double((long long)(1023 - 52 + eu) << 52);  // 2^(e - 52)
        double m = s * sc;
        int L = T.lmax;
        auto entry = [&](int cc, int l) -> cdouble* {  // block (cc, level l) of binade eu
          return l == 0 ? (cdouble*)(tab + (size_t)(eu - emin) * nstride + cc)
                        : (cdouble*)(T.p + T.off[l] + (size_t)(eu - emin) * T.nb[l] + (cc >> l));
        };
        auto step = [&](double d0, double dd) {  // m after the block, if no lane leaves the binade
          return m + __builtin_fma((double)(__double2loint(m) & 1), dd, d0);
        };
        while (c < fast_hi) {  // uniform
          int Lc = min(L, 31 - __clz(fast_hi - c));
          if (c) Lc = min(Lc, __ffs(c) - 1);
          cdouble* tb = entry(c, Lc);
          const double d0 = tb[0], dd = tb[1];
          const double mn = step(d0, dd);
          if (__builtin_amdgcn_ballot_w64(!(mn > -TWO53)) == 0ull) { m = mn; c += 1 << Lc; L = T.lmax; continue; }
          if (Lc == 0) break;
          if (!wdesc || Lc < 2) { L = Lc - 1; continue; }
          // a crossing inside [c, c + 2^Lc): the next two levels of the halving search from one
          // round trip -- (c, Lc - 1), then (c + 2^(Lc-1), Lc - 2) after a success or (c, Lc - 2)
          // after a failure, the same blocks in the same order as one level at a time
          const int l1 = Lc - 1, l2 = Lc - 2;
          cdouble* ta = entry(c, l1);
          cdouble* tbs = entry(c + (1 << l1), l2);
          cdouble* tcf = entry(c, l2);
          const double a0 = ta[0], ad = ta[1], b0 = tbs[0], bd = tbs[1], f0 = tcf[0], fd = tcf[1];
          const double ma = step(a0, ad);
          if (__builtin_amdgcn_ballot_w64(!(ma > -TWO53)) == 0ull) {
            m = ma; c += 1 << l1;
            const double mb = step(b0, bd);
            if (__builtin_amdgcn_ballot_w64(!(mb > -TWO53)) == 0ull) { m = mb; c += 1 << l2; L = T.lmax; continue; }
          } else {
            const double mf = step(f0, fd);
            if (__builtin_amdgcn_ballot_w64(!(mf > -TWO53)) == 0ull) { m = mf; c += 1 << l2; L = T.lmax; continue; }
          }
          if (l2 == 0) break;
          L = l2 - 1;
        }
        s = m * isc;
        if (c >= fast_hi) continue;
      } else if (eu >= emin && eu < emin + ne && __builtin_amdgcn_ballot_w64(!(s < 0.0) || e != eu) == 0ull) {
        const int gn = min(WCG, fast_hi - c);
        // uniform address, read-only for the kernel's life: through the constant address space, so
        // that the group's entries are scalar loads (registers shared by the wave; no texture path)
        typedef const __attribute__((address_space(4))) double cdouble;
        cdouble* tb = (cdouble*)(tab + (size_t)(eu - emin) * nstride + c);  // the padding covers c + WCG
        double d0[WCG], dd[WCG];
#pragma unroll
        for (int k = 0; k < WCG; k++) { d0[k] = tb[2 * k]; dd[k] = tb[2 * k + 1]; }
        const double sc = __longlong_as_double((long long)(1023 + 52 - eu) << 52);   // 2^(52 - e)
        const double isc = __longlong_as_double((long long)(1023 - 52 + eu) << 52);  // 2^(e - 52)
        double m = s * sc;  // an integer, |m| in [2^52, 2^53): its last mantissa bit is its parity
        int j = gn;
        bool run = true;
#pragma unroll
        for (int k = 0; k < WCG; k++) {
          if (run && k < gn) {  // uniform
            const double mn = m + __builtin_fma((double)(__double2loint(m) & 1), dd[k], d0[k]);
            if (__builtin_amdgcn_ballot_w64(!(mn > -TWO53))) { j = k; run = false; }  // leaves the binade, or NaN
            else m = mn;
          }
        }
        s = m * isc;
        c += j;
        if (j == gn) continue;
      }
    }
    // the general step for chunk c
    const int cb = c * WC;
    const int lo = max(ws - cb, 0), hi = min(end - cb, WC);  // the lane's sites of the chunk: [lo, hi)
    bool need = lo < hi;
    if (need && lo == 0 && hi == WC && s < 0.0) {
      const int e = (int)((__double_as_longlong(s) >> 52) & 0x7FF) - 1023;
      if (e >= emin && e < emin + ne) {
        const double2 d = tab[(size_t)(e - emin) * nstride + c];
        const double sc = __longlong_as_double((long long)(1023 + 52 - e) << 52);
        const double isc = __longlong_as_double((long long)(1023 - 52 + e) << 52);
        const double m = s * sc;
        const double mn = m + __builtin_fma((double)(__double2loint(m) & 1), d.y, d.x);
        if (mn > -TWO53) { s = mn * isc; need = false; }
      }
    }
    if (__builtin_amdgcn_ballot_w64(need)) {
      const double v = nullrow[pr[phys((uint32_t)(cb + lane))].y];  // cb + 63 is inside the padded array
      const int2 vv = make_int2(__double2loint(v), __double2hiint(v));
#pragma unroll 8
      for (int q = 0; q < WC; q++) {
        const double x = __hiloint2double(__builtin_amdgcn_readlane(vv.y, q), __builtin_amdgcn_readlane(vv.x, q));
        if (need && q >= lo && q < hi) s += x;
      }
    }
    c++;
  }
  if (valid) out[ws] = s;
}

// one trial's rows into the (position, row) array: pr[phys(i)].y = row[i] + 1 (device row), read
// straight from the pinned host staging (no copy-engine transfer, which would order this
// stream's work behind other streams' copies); block 0 also takes the whole-chromosome null
// sums.  row == null: the uploaded rows (pr0).  T: the staging's row width (1, 2 or 4 bytes:
// the narrowest that holds the table's rows, so that the PCIe reads are as few as can be).
template <typename T>
__global__ void __launch_bounds__(64) scatter_rows_kernel(uint2* __restrict__ pr, const T* __restrict__ row,
                                                          const uint2* __restrict__ pr0, int n,
                                                          double* __restrict__ chr_null,
                                                          const double* __restrict__ chr_null_src, int n_chr) {
  // One wave per block and no LDS, so that its blocks fit beside two resident search
  // workgroups on a CU (they hold the whole LDS and 6 of the 8 wave slots per SIMD): an LDS-tiled
  // version waited for search workgroups to retire, 137 us per C4 trial at ~7 GB/s, although the
  // PCIe read itself takes ~30 us (HISTORY.md, hostread_probe).  A block takes 64 * E
  // sites: one 16-B read of the pinned host rows per lane (few, wide PCIe reads), then the wave
  // transposes them by shuffles so that each store k covers 64 consecutive sites.
  constexpr int E = 16 / sizeof(T);
  const int l = threadIdx.x, base = blockIdx.x * 64 * E;
  if (row) {
    union { uint4 v; T t[E]; } u;
    u.v = make_uint4(0u, 0u, 0u, 0u);
    const int i = base + E * l;
    if (i + E <= n) u.v = *reinterpret_cast<const uint4*>(row + i);
    else
      for (int k = 0; k < E; k++) if (i + k < n) u.t[k] = row[i + k];
    // site base + 64 k + l sits in lane (64 k + l) / E, element l % E (E divides 64)
    const int idx = l % E, dw = idx * (int)sizeof(T) / 4, sh = (idx * (int)sizeof(T) % 4) * 8;
#pragma unroll
    for (int k = 0; k < E; k++) {
      const int src = (64 * k + l) / E;
      const unsigned w0 = (unsigned)__shfl((int)u.v.x, src, 64), w1 = (unsigned)__shfl((int)u.v.y, src, 64);
      const unsigned w2 = (unsigned)__shfl((int)u.v.z, src, 64), w3 = (unsigned)__shfl((int)u.v.w, src, 64);
      const unsigned w = dw == 0 ? w0 : dw == 1 ? w1 : dw == 2 ? w2 : w3;
      const unsigned r = sizeof(T) == 4 ? w : (w >> sh) & (unsigned)((1ull << (8 * sizeof(T))) - 1ull);
      const int q = base + 64 * k + l;
      if (q < n) pr[phys(q)].y = r + 1u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < E; k++) {
      const int q = base + 64 * k + l;
      if (q < n) pr[phys(q)].y = pr0[phys(q)].y;
    }
  }
  if (blockIdx.x == 0 && chr_null_src)
    for (int c = l; c < n_chr; c += 64) chr_null[c] = chr_null_src[c];
}

// A trial's block plan (fsclg_slot_set_rows_plan, scan-chromosome.c:336-389 on the device): the
// slot's rows start as the uploaded ones (scatter_rows_kernel, row == null), then each group of
// the plan is applied in turn.  A group's entries touch disjoint sites: one workgroup per kind-0
// entry (<= 4096 sites, perm.c) swaps rows[i + t] <-> rows[j + t] in the row words of the
// interleaved (position, row) array; the reads of a thread complete before its writes, and no
// other thread of the launch touches those sites.  The row array of one slot is only written by
// the upload stream, in stream order.
__global__ void __launch_bounds__(256) plan_swap_kernel(uint2* __restrict__ pr, const fsclg_swap_t* __restrict__ ent,
                                                        int e0) {
  // a thread's sites of both ranges are loaded three at a time before they are stored: one memory
  // latency per 768 sites of the entry instead of one per 256 (the stores may alias the next loads
  // as far as the compiler can tell, so a load-store loop waits for each round trip); three keep the
  // kernel within the 32 registers the search waves leave free
#ifndef FSCLG_SWAP_PER
#define FSCLG_SWAP_PER 3
#endif
  constexpr int PER = FSCLG_SWAP_PER;
  const fsclg_swap_t x = ent[e0 + blockIdx.x];
  char* rw = reinterpret_cast<char*>(pr) + 4;  // the row words; 32-bit byte offsets (scalar base + vector offset)
  auto row = [rw](uint32_t i) -> uint32_t& { return *reinterpret_cast<uint32_t*>(rw + (phys(i) << 3)); };
  for (int t0 = threadIdx.x; t0 < x.len; t0 += 256 * PER) {
    uint32_t va[PER], vb[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int t = t0 + 256 * k;
      if (t < x.len) {
        va[k] = row((uint32_t)(x.i + t));
        vb[k] = row((uint32_t)(x.j + t));
      }
    }
#pragma unroll
    for (int k = 0; k < PER; k++) {
      const int t = t0 + 256 * k;
      if (t < x.len) {
        row((uint32_t)(x.i + t)) = vb[k];
        row((uint32_t)(x.j + t)) = va[k];
      }
    }
  }
}

// kind 1, a block whose source and target overlap (d = |i - j| < len): the reference's element
// swaps in order rotate [lo, lo + len + d), out[lo + t] = in[lo + d + t] for t < len and
// in[lo + t % d] after; through a copy of the range (two launches: all reads before any write)
__global__ void __launch_bounds__(256) plan_rot_save_kernel(const uint2* __restrict__ pr, uint32_t* __restrict__ tmp,
                                                            int lo, int R) {
  for (int t = blockIdx.x * 256 + threadIdx.x; t < R; t += gridDim.x * 256) tmp[t] = pr[phys((uint32_t)(lo + t))].y;
}

__global__ void __launch_bounds__(256) plan_rot_kernel(uint2* __restrict__ pr, const uint32_t* __restrict__ tmp,
                                                       int lo, int len, int d) {
  for (int t = blockIdx.x * 256 + threadIdx.x; t < len + d; t += gridDim.x * 256)
    pr[phys((uint32_t)(lo + t))].y = tmp[t < len ? d + t : t % d];
}

}  // namespace

// ----------------------------------------------------------------- host shim
constexpr int NSLOT = FSCLG_N_SLOTS;
constexpr int NBATCH = FSCLG_N_BATCHES;

// FSCLG_HOST_PROFILE=1 (development aid): host seconds in the shim's submit-side calls, printed to stderr at
// fsclg_close: [0] fsclg_slot_windows, [1] waits for a slot's previous window launch, [2] fsclg_search_submit,
// [3] its launches (the HIP calls), [4] its window check (ensure_windows)
static double g_hprof[12];
static double hnow() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static bool hprof_on() { static const bool on = getenv("FSCLG_HOST_PROFILE") != nullptr; return on; }


// one trial's rows on the device (fsclg_slot_set_rows): the (position, row) array, the
// whole-chromosome null sums and the per-window null sums of those rows
struct Slot {
  uint2* d_pr = nullptr;          // (biased position, device row), n_snps + PAD
  double* d_chr_null = nullptr;
  double* d_win_null = nullptr;   // [n_snps], valid for (win_er, rows) while win_valid
  int win_er = -1;
  bool win_valid = false;         // win_null holds every window start, or (win_part) the ranges wdone
  bool win_part = false;
  std::vector<int2> wdone;        // window starts [x, y) summed for the slot's rows, sorted, disjoint
  int2* p_wtasks = nullptr;       // pinned: the tasks of the slot's last partial window launch
  int wtask_cap = 0;
  uint32_t* h_rows = nullptr;     // pinned (coherent) staging of one trial's rows, read by scatter_rows_kernel
  double* h_null = nullptr;       // pinned (coherent) whole-chromosome null sums, n_chr
  int rows_cap = 0, null_cap = 0;
  hipEvent_t ready = nullptr;     // recorded on the upload stream after the slot's last upload
  hipEvent_t wev0 = nullptr, wev1 = nullptr;  // bracket the slot's last window null-sum launch
  bool wpend = false;             // its time not yet added to window_ms (read without blocking later)
  int users = 0;                  // batches submitted on this slot and not yet waited for
  double2* d_ctab = nullptr;      // chunk_table_kernel's table for the slot's rows (window_chunk_kernel)
  double2* d_ctree = nullptr;     // chunk_tree_kernel's block maps over it
  size_t ctree_cap = 0;
  CTree ctree = {};
  size_t ctab_cap = 0;            // entries
  bool ctab_valid = false;        // built for the slot's rows with (ctab_emin, ctab_ne)
  int ctab_emin = 0, ctab_ne = 0;
};

// one search_maxpos launch group (fsclg_search_submit / fsclg_search_wait): its stream,
// events, device and pinned host buffers, and the host-side dedup / ordering of its cells
struct Batch {
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // bracket the kernels
  hipEvent_t ev2 = nullptr;                  // after the results' D2H
  // the kernels read their inputs from and write their outputs to pinned coherent host memory
  // (a few bytes per workgroup): no copy-engine transfers on the batch streams, which would
  // order one stream's kernels behind another stream's copies and serialise the trials
  fsclg_cell_t* p_cells = nullptr;
  fsclg_point_t* p_out = nullptr;
  int cap = 0;
  fsclg_point_t* d_ept = nullptr;   // endpoint results: written by one launch, read by the next
  int2* p_epos = nullptr;
  int2* p_cell_ep = nullptr;
  int ept_cap = 0, pep_cap = 0, pcep_cap = 0;
  unsigned long long* p_ctrace = nullptr;  // FSCLG_CELL_TRACE=<file>: per-cell timing appended per launch
  int ctrace_cap = 0;
  int trace_n = 0;                  // cells of the traced launch (the event area follows them)
  unsigned long long* ivhist = nullptr;    // this launch measures the interval histogram (FSCLG_IVHIST)
  bool traced = false;
  std::vector<int> uidx, upos, order, sidx;
  cellorder::RangeMemo<fsclg_cell_t, int2> wr_memo;  // its cells' window ranges at the last submit
  std::vector<unsigned long long> ekeys;
  std::vector<fsclg_cell_t> ucells;
  std::vector<int2> epos, ucell_ep;
  int n_cells = 0, nu = 0, nlaunch = 0, slot = -1;
  bool pending = false;
  int split_max = 1;                // fsclg_set_batch_split
  int split = 1;                    // members per cell of the current launch
  int eval_range = 0, bp_resl = 0;  // of the submitted launch (a split launch re-run unsplit)
  char* d_xacc = nullptr;           // split cells' accumulators and arrival counters
  unsigned int* d_xcnt = nullptr;
  size_t xacc_cap = 0;
  int xcnt_cap = 0;
};

struct fsclg_ctx {
  int device;
  hipStream_t ustream;            // uploads (rows, null sums, window sums), high priority
  hipStream_t bstream[3];         // batches 0-1: high priority; even / odd batches 2..: normal
  hipEvent_t ev_ref;              // time origin of the busy intervals (fsclg_reset_stats)
  hipEvent_t wev0, wev1;          // window null-sum kernel timing
  // tables
  double* d_logt = nullptr;
  double* d_lx = nullptr;         // FSCLG_LOG_CALC: logx_mid's table (LX_BYTES)
  int lx_on = 0;
  double* d_coef = nullptr;
  double* d_null = nullptr;
  double* d_thr = nullptr;
  int n_rows = 0, n_iv = 0;
  double step = 0.0;
  // snps
  uint2* d_pr0 = nullptr;         // (biased position, device row) with the unpermuted rows
  uint32_t* d_plan_tmp = nullptr; // fsclg_slot_set_rows_plan: the range of an overlapping block
  int plan_tmp_cap = 0;
  std::vector<uint2> h_pr0;
  int n_snps = 0;
  int32_t* d_chr_start = nullptr;
  int32_t* d_chr_n = nullptr;
  int2* d_wtasks = nullptr;
  int n_wtasks = 0, wtask_cap = 0, wtask_er = -1;
  int wtask_chunk = -1;                 // the dense task list is for window_chunk_kernel (256 per task) or not
  std::vector<double> h_nullrows;       // the uploaded null rows (chunk_params)
  double window_ms = 0.0;
  int n_chr = 0;
  std::vector<int> h_chr_n;
  std::vector<int32_t> h_pos, h_chr_start;
  cellorder::SiteIndex site_index;  // window_ranges' searches (built on first use after an upload)
  bool sidx_valid = false;
  long long site_epoch = 0;         // site uploads indexed so far (window_ranges' memo key)
  cellorder::RangeMemo<fsclg_cell_t, int2> wr_memo;
  std::vector<int2> wr_need;
  std::vector<int> wr_idx;
  int lt_hi = 0;                        // logt3 branch-2 entries [256, lt_hi) staged in LDS
  std::vector<long long> h_row_cnt;     // sites per device row
  std::vector<double> h_lt3;
  Slot slot[NSLOT];
  Batch batch[NBATCH];
  // LDS coefficient cache plan (fsclg_plan_cache)
  bool plan_dirty = true;
  bool hist_pending = false;          // the next search_maxpos launch measures the interval histogram
  unsigned long long* d_ivhist = nullptr;
  int ivhist_n = 0;
  int c_ivc0 = 0, c_civ = 0, c_crow = 0;
  double c_cover = 0.0;
  int c_ivc0_b = 0, c_civ_b = 0;         // the window beside band mode's BandLds (Params::off_bd)
  double c_cover_b = 0.0;
  // alpha grid
  std::vector<double> h_coarse, h_refine;
  std::vector<int32_t> h_nref;
  uint32_t* d_dfail = nullptr;     // walk thresholds of the alpha grid (Params::dfail)
  uint32_t* d_dband = nullptr;     // band cuts of the alpha grid (Params::dband)
  int32_t* d_tpos = nullptr;       // position of every 128th site (Params::tpos)
  std::vector<double> h_thr;       // the interval thresholds (Params::thr)
  double* d_la_coarse = nullptr;
  double* d_la_refine = nullptr;
  int32_t* d_n_refine = nullptr;
  int n_coarse = 0;
  unsigned long long* d_stats = nullptr;
  std::unordered_map<unsigned long long, uint32_t> cell_cost;  // (chr, start, end) -> cost of its last run
  unsigned long long n_dup_cells = 0, n_ep_saved = 0;
  unsigned long long n_split_retry = 0;
  unsigned long long ci_count[16] = {0};  // results' coarse alpha index (nearest coarse grid value): the guess
  int ci_guess = 5;                       // of split cells' speculative refine walks (Params::ci_guess)
  double kernel_ms = 0.0;
  unsigned long long launches = 0;
  std::vector<std::pair<double, double>> busy;  // [start, end) ms of each batch's kernels since ev_ref
};

static thread_local char g_err[512];
static int set_err(int code, const char* what, hipError_t e = hipSuccess) {
  if (e != hipSuccess) snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
  else snprintf(g_err, sizeof g_err, "%s", what);
  return code;
}
#define HIPCHK(x, what) do { hipError_t e_ = (x); if (e_ != hipSuccess) return set_err(FSCLG_E_HIP, what, e_); } while (0)

template <typename T>
static int upload(T** dst, const T* src, size_t n, hipStream_t s) {
  if (*dst) { hipFree(*dst); *dst = nullptr; }
  hipError_t e = hipMalloc((void**)dst, sizeof(T) * (n ? n : 1));
  if (e != hipSuccess) return set_err(FSCLG_E_HIP, "hipMalloc", e);
  if (n && src) {
    e = hipMemcpyAsync(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return set_err(FSCLG_E_HIP, "hipMemcpyAsync", e);
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return set_err(FSCLG_E_HIP, "hipStreamSynchronize", e);
  }
  return FSCLG_OK;
}

static int update_dfail(fsclg_ctx* c);
static int update_dband(fsclg_ctx* c);

// least double x with (int)((x - LOG_AD_MIN) / step) >= j (sm-spline.c:52), by bisection over the
// ordered doubles; the host evaluates the reference's expression with IEEE division
static long long dkey(double x) { long long b; memcpy(&b, &x, 8); return b < 0 ? -(b & 0x7fffffffffffffffll) : b; }
static double dval(long long k) { long long b = k < 0 ? ((-k) | (long long)0x8000000000000000ull) : k; double x; memcpy(&x, &b, 8); return x; }
static int ref_interval(double x, double step) { return (int)((x - LOG_AD_MIN) / step); }
static double interval_threshold(int j, double step) {
  long long lo = dkey(LOG_AD_MIN - 1.0), hi = dkey(LOG_AD_MAX + 64.0);
  if (ref_interval(dval(hi), step) < j) return dval(hi);
  while ((unsigned long long)hi - (unsigned long long)lo > 1) {  // invariant: f(lo) < j <= f(hi)
    const long long m = lo + (long long)(((unsigned long long)hi - (unsigned long long)lo) / 2);
    if (ref_interval(dval(m), step) >= j) hi = m; else lo = m;
  }
  return dval(hi);
}

extern "C" {

const char* fsclg_last_error(void) { return g_err; }

int fsclg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int fsclg_open(int device, fsclg_ctx** out) {
  if (!out) return set_err(FSCLG_E_ARG, "null out");
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (device < 0 || device >= n) return set_err(FSCLG_E_ARG, "no such device");
  HIPCHK(hipSetDevice(device), "hipSetDevice");
  fsclg_ctx* c = new fsclg_ctx();
  c->device = device;
  // the rand-stream critical batches (and the uploads they wait for) get the high-priority
  // streams: their workgroups take the next free slots ahead of the bulk of a trial
  int lo = 0, hi = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
  HIPCHK(hipStreamCreateWithPriority(&c->ustream, hipStreamNonBlocking, hi), "hipStreamCreate");
  // FSCLG_RESERVE=r (experiment): the bulk streams leave every r-th CU to the blocking batch's
  // high-priority stream (r = 4: a quarter of the CUs), whose workgroups then find free slots
  const int reserve = getenv("FSCLG_RESERVE") ? atoi(getenv("FSCLG_RESERVE")) : 0;
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  for (int k = 0; k < 3; k++) {
    if (k > 0 && reserve > 1) {
      std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
      for (int cu = 0; cu < prop.multiProcessorCount; cu++)
        if (cu % reserve != reserve - 1) mask[cu / 32] |= 1u << (cu % 32);
      HIPCHK(hipExtStreamCreateWithCUMask(&c->bstream[k], (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
    } else {
      HIPCHK(hipStreamCreateWithPriority(&c->bstream[k], hipStreamNonBlocking, k == 0 ? hi : lo), "hipStreamCreate");
    }
  }
  for (int b = 0; b < NBATCH; b++) {
    Batch& B = c->batch[b];
    B.stream = c->bstream[b < 2 ? 0 : 1 + (b & 1)];
    HIPCHK(hipEventCreate(&B.ev0), "hipEventCreate");
    HIPCHK(hipEventCreate(&B.ev1), "hipEventCreate");
    HIPCHK(hipEventCreateWithFlags(&B.ev2, hipEventDisableTiming), "hipEventCreate");
  }
  for (int s = 0; s < NSLOT; s++) {
    HIPCHK(hipEventCreateWithFlags(&c->slot[s].ready, hipEventDisableTiming), "hipEventCreate");
    HIPCHK(hipEventCreate(&c->slot[s].wev0), "hipEventCreate");
    HIPCHK(hipEventCreate(&c->slot[s].wev1), "hipEventCreate");
  }
  HIPCHK(hipEventCreate(&c->ev_ref), "hipEventCreate");
  HIPCHK(hipEventCreate(&c->wev0), "hipEventCreate");
  HIPCHK(hipEventCreate(&c->wev1), "hipEventCreate");
  HIPCHK(hipMalloc((void**)&c->d_stats, sizeof(unsigned long long) * 24), "hipMalloc stats");  // 8 + FSCLG_TRIP_STAMPS
  HIPCHK(hipMemset(c->d_stats, 0, sizeof(unsigned long long) * 24), "hipMemset");
  HIPCHK(hipEventRecord(c->ev_ref, c->ustream), "hipEventRecord");
  HIPCHK(hipEventSynchronize(c->ev_ref), "hipEventSynchronize");
  *out = c;
  return FSCLG_OK;
}

int fsclg_close(fsclg_ctx* c) {
  if (!c) return FSCLG_OK;
  if (hprof_on())
    fprintf(stderr, "fsclg host profile: slot_windows %.3f s (window waits %.3f s, ranges %.3f s, partial launch "
                    "%.3f s), search_submit %.3f s (launches %.3f s, window check %.3f s, dedup + endpoints %.3f s, "
                    "order %.3f s)\n", g_hprof[0], g_hprof[1], g_hprof[5], g_hprof[6], g_hprof[2], g_hprof[3], g_hprof[4],
            g_hprof[7], g_hprof[8]);
  hipSetDevice(c->device);
  hipDeviceSynchronize();
  void* ptrs[] = {c->d_ivhist, c->d_logt, c->d_coef, c->d_null, c->d_thr, c->d_pr0,
                  c->d_chr_start, c->d_chr_n, c->d_wtasks, c->d_la_coarse, c->d_la_refine, c->d_n_refine,
                  c->d_stats, c->d_dfail, c->d_dband, c->d_tpos, c->d_plan_tmp, c->d_lx};
  for (void* p : ptrs) if (p) hipFree(p);
  for (Slot& S : c->slot) {
    for (void* p : {(void*)S.d_pr, (void*)S.d_chr_null, (void*)S.d_win_null, (void*)S.d_ctab, (void*)S.d_ctree})
      if (p) hipFree(p);
    for (void* p : {(void*)S.h_rows, (void*)S.h_null, (void*)S.p_wtasks}) if (p) hipHostFree(p);
    hipEventDestroy(S.ready);
    if (S.wev0) hipEventDestroy(S.wev0);
    if (S.wev1) hipEventDestroy(S.wev1);
  }
  for (Batch& B : c->batch) {
    if (B.d_ept) hipFree(B.d_ept);
    if (B.d_xacc) hipFree(B.d_xacc);
    if (B.d_xcnt) hipFree(B.d_xcnt);
    for (void* p : {(void*)B.p_cells, (void*)B.p_out, (void*)B.p_epos, (void*)B.p_cell_ep, (void*)B.p_ctrace})
      if (p) hipHostFree(p);
    hipEventDestroy(B.ev0);
    hipEventDestroy(B.ev1);
    hipEventDestroy(B.ev2);
  }
  for (hipStream_t st : c->bstream) hipStreamDestroy(st);
  hipEventDestroy(c->ev_ref);
  hipEventDestroy(c->wev0);
  hipEventDestroy(c->wev1);
  hipStreamDestroy(c->ustream);
  delete c;
  return FSCLG_OK;
}

static bool any_pending(const fsclg_ctx* c) {
  for (const Batch& B : c->batch) if (B.pending) return true;
  return false;
}

#if FSCLG_LOG_CALC
// logx_mid's table: per k, log(c) as hi + lo (long double) and RN(1/c); then every entry of the
// mid branch evaluated here with the device's operations, and the lo part of a k whose entries
// do not all reproduce the reference's table shifted (in 2^-68 steps, up to 2^-59) until they do;
// then the device's own evaluation checked once against the uploaded table.  Any entry still
// off: the mid branch keeps the gather (lx_on 0).
static int logx_setup(fsclg_ctx* c, const std::vector<double>& lt3) {
  std::vector<double> lx(LX_BYTES / 8, 0.0);
  for (int k = 0; k < 256; k++) {
    const double cc = (256.0 + k) * 128.0;
    const long double lc = logl((long double)cc);
    lx[4 * k] = (double)lc;
    lx[4 * k + 1] = (double)(lc - (long double)lx[4 * k]);
    lx[4 * k + 2] = 1.0 / cc;
  }
  auto k_of = [](uint32_t i) { return ((i << (15 - (31 - __builtin_clz(i)))) >> 7) & 255u; };
  auto k_ok = [&](uint32_t k) {
    for (uint32_t i = 256; i < 0x10000u; i++)
      if (k_of(i) == k && logx_mid(i, lx.data()) != lt3[0x10000u + i]) return false;
    return true;
  };
  std::vector<char> bad_k(256, 0);
  for (uint32_t i = 256; i < 0x10000u; i++)
    if (logx_mid(i, lx.data()) != lt3[0x10000u + i]) bad_k[k_of(i)] = 1;
  bool ok = true;
  for (int k = 0; k < 256 && ok; k++) {
    if (!bad_k[k]) continue;
    const double base = lx[4 * k + 1];
    bool fixed = false;
    for (int t = 1; t <= 512 && !fixed; t++)
      for (int sg = -1; sg <= 1 && !fixed; sg += 2) {
        lx[4 * k + 1] = base + sg * t * 0x1p-68;
        fixed = k_ok((uint32_t)k);
      }
    if (!fixed) { lx[4 * k + 1] = base; ok = false; }
  }
  c->lx_on = 0;
  if (!ok) return FSCLG_OK;
  int r;
  if ((r = upload(&c->d_lx, lx.data(), lx.size(), c->ustream))) return r;
  unsigned long long* d_bad = nullptr;
  unsigned long long bad = 1;
  HIPCHK(hipMalloc((void**)&d_bad, sizeof bad), "hipMalloc");
  HIPCHK(hipMemsetAsync(d_bad, 0, sizeof bad, c->ustream), "hipMemsetAsync");
  hipLaunchKernelGGL(logx_check_kernel, dim3((0x10000 - 256 + 255) / 256), dim3(256), 0, c->ustream, c->d_lx, c->d_logt,
                     d_bad);
  HIPCHK(hipGetLastError(), "launch logx_check_kernel");
  HIPCHK(hipMemcpyAsync(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost, c->ustream), "hipMemcpyAsync");
  HIPCHK(hipStreamSynchronize(c->ustream), "hipStreamSynchronize");
  hipFree(d_bad);
  c->lx_on = bad == 0 && !getenv("FSCLG_NO_LOGX");
  if (bad) fprintf(stderr, "fsclg: the device's mid-branch log distances differ from the table in %llu entries: "
                           "the table is gathered instead\n", bad);
  return FSCLG_OK;
}
#endif

int fsclg_upload_tables(fsclg_ctx* c, const double* log_table, const double* coef, int n_rows, int n_iv,
                        const double* nullrow, double log_ad_step) {
  if (!c || !log_table || !coef || !nullrow || n_rows <= 0 || n_iv <= 0) return set_err(FSCLG_E_ARG, "tables");
  if ((unsigned long long)(n_rows + 1) * (unsigned long long)n_iv * 32ull >= (1ull << 32))
    return set_err(FSCLG_E_ARG, "coefficient table exceeds 4 GiB (32-bit offsets)");
  if (any_pending(c)) return set_err(FSCLG_E_STATE, "search batches in flight");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  // the three branches of sm-search.c:40-46 (c_b + log_table[i]) as one table; the same
  // IEEE double add as the reference's, so every entry is bit-identical to its result
  std::vector<double> lt3(3 * 0x10000);
  const double cb[3] = {0.0, 5.545177444479562, 11.783502069519070};
  for (int b = 0; b < 3; b++)
    for (int i = 0; i < 0x10000; i++) {
      volatile double v = cb[b] + log_table[i];
      lt3[(size_t)b * 0x10000 + i] = b ? (double)v : log_table[i];
    }
  if ((r = upload(&c->d_logt, lt3.data(), lt3.size(), c->ustream))) return r;
#if FSCLG_LOG_CALC
  if ((r = logx_setup(c, lt3))) return r;
#endif
  c->h_lt3.swap(lt3);
  if ((r = update_dfail(c))) return r;
  // [row][iv][4] -> [iv][plane][1 + row][2] (coef_off): device row 0 is an all-zero sentinel
  // (terms exactly 0); plane 0 holds (c0, c1), plane 1 (c2, c3)
  const size_t stride = (size_t)n_rows + 1;
  std::vector<double> tcoef(stride * n_iv * 4, 0.0);
  for (int rr = 0; rr < n_rows; rr++)
    for (int iv = 0; iv < n_iv; iv++)
      for (int pl = 0; pl < 2; pl++)
        memcpy(&tcoef[(((size_t)iv * 2 + pl) * stride + rr + 1) * 2], coef + ((size_t)rr * n_iv + iv) * 4 + 2 * pl,
               sizeof(double) * 2);
  if ((r = upload(&c->d_coef, tcoef.data(), tcoef.size(), c->ustream))) return r;
  std::vector<double> nul(1, 0.0);
  nul.insert(nul.end(), nullrow, nullrow + n_rows);
  if ((r = upload(&c->d_null, nul.data(), nul.size(), c->ustream))) return r;
  c->h_nullrows = nul;
  std::vector<double> thr((size_t)n_iv + 1, 0.0);
  for (int j = 1; j < n_iv; j++) thr[j] = interval_threshold(j, log_ad_step);
  thr[0] = -__builtin_inf();     // iv 0 never steps down
  thr[n_iv] = __builtin_inf();   // iv n_iv-1 never steps up (the reference clamps)
  if ((r = upload(&c->d_thr, thr.data(), thr.size(), c->ustream))) return r;
  c->n_rows = n_rows; c->n_iv = n_iv; c->step = log_ad_step;
  c->h_thr = thr;
  if ((r = update_dband(c))) return r;
  c->plan_dirty = true;
  for (Slot& S : c->slot) { S.win_valid = false; S.ctab_valid = false; }
  return FSCLG_OK;
}

int fsclg_upload_snps(fsclg_ctx* c, const int32_t* pos, const uint32_t* row, int n_snps,
                      const int32_t* chr_start, const int32_t* chr_n, int n_chr) {
  if (!c || !pos || !row || n_snps <= 0 || !chr_start || !chr_n || n_chr <= 0) return set_err(FSCLG_E_ARG, "snps");
  if (any_pending(c)) return set_err(FSCLG_E_STATE, "search batches in flight");
  for (int i = 0; i < n_chr; i++)
    if (chr_start[i] < 0 || chr_n[i] <= 0 || chr_start[i] + chr_n[i] > n_snps) return set_err(FSCLG_E_ARG, "chr limits");
  for (int i = 0; i < n_snps; i++)
    if (c->n_rows && row[i] >= (uint32_t)c->n_rows) return set_err(FSCLG_E_ARG, "row index out of table");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  // interleaved per 128-site block (phys), rounded up to whole blocks, then PAD slack (zeros:
  // a valid position and row, never counted)
  std::vector<uint2> pr(((size_t)n_snps + 127) / 128 * 128 + PAD, make_uint2(POS_BIAS, 0u));
  for (int i = 0; i < n_snps; i++) pr[phys((uint32_t)i)] = make_uint2((uint32_t)pos[i] ^ POS_BIAS, row[i] + 1);
  if ((r = upload(&c->d_pr0, pr.data(), pr.size(), c->ustream))) return r;
  {  // band cut searches: the position of the first site of every 128-site block
    std::vector<int32_t> tp(((size_t)n_snps + 127) / 128);
    for (size_t t = 0; t < tp.size(); t++) tp[t] = pos[t * 128];
    if ((r = upload(&c->d_tpos, tp.data(), tp.size(), c->ustream))) return r;
  }
  for (Slot& S : c->slot) {
    if ((r = upload(&S.d_pr, pr.data(), pr.size(), c->ustream))) return r;
    if ((r = upload<double>(&S.d_chr_null, nullptr, (size_t)n_chr, c->ustream))) return r;
    if ((r = upload<double>(&S.d_win_null, nullptr, (size_t)n_snps, c->ustream))) return r;
    S.win_valid = false; S.win_er = -1; S.ctab_valid = false;
    HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");
  }
  c->n_snps = n_snps;
  if ((r = upload(&c->d_chr_start, chr_start, (size_t)n_chr, c->ustream))) return r;
  if ((r = upload(&c->d_chr_n, chr_n, (size_t)n_chr, c->ustream))) return r;
  c->wtask_er = -1;
  c->n_snps = n_snps; c->n_chr = n_chr;
  c->h_chr_n.assign(chr_n, chr_n + n_chr);
  c->h_chr_start.assign(chr_start, chr_start + n_chr);
  c->h_pos.assign(pos, pos + n_snps);
  c->sidx_valid = false;
  c->cell_cost.clear();
  {  // |d| of a walk stays within a chromosome's span (plus grid slack): branch-2 index range
    long long span = 0;
    for (int i = 0; i < n_chr; i++)
      span = std::max(span, (long long)pos[chr_start[i] + chr_n[i] - 1] - (long long)pos[chr_start[i]]);
    c->lt_hi = getenv("FSCLG_NO_LTLDS") ? 0 : (int)std::min(32768ll, std::max(256ll, (span >> 16) + 64));
    if (c->lt_hi <= 256) c->lt_hi = 0;
  }
  c->h_row_cnt.clear();
  for (int i = 0; i < n_snps; i++) {
    const uint32_t dr = row[i] + 1;
    if (dr >= c->h_row_cnt.size()) c->h_row_cnt.resize(dr + 1, 0);
    c->h_row_cnt[dr]++;
  }
  c->h_pr0.swap(pr);
  c->plan_dirty = true;
  return FSCLG_OK;
}

// pinned host memory the kernels read or write directly (coherent: no cache flush needed
// between a kernel's stores and the host's reads after its completion event)
static constexpr unsigned HOSTMEM = hipHostMallocCoherent | hipHostMallocMapped;

static int ensure_null_staging(fsclg_ctx* c, Slot& S) {
  if (S.null_cap >= c->n_chr) return FSCLG_OK;
  if (S.h_null) hipHostFree(S.h_null);
  S.h_null = nullptr; S.null_cap = 0;
  HIPCHK(hipHostMalloc((void**)&S.h_null, sizeof(double) * c->n_chr, HOSTMEM), "hipHostMalloc null sums");
  S.null_cap = c->n_chr;
  return FSCLG_OK;
}

static int ensure_row_staging(fsclg_ctx* c, Slot& S) {
  int r;
  if ((r = ensure_null_staging(c, S))) return r;
  if (S.rows_cap >= c->n_snps) return FSCLG_OK;
  if (S.h_rows) hipHostFree(S.h_rows);
  S.h_rows = nullptr; S.rows_cap = 0;
  HIPCHK(hipHostMalloc((void**)&S.h_rows, sizeof(uint32_t) * c->n_snps, HOSTMEM), "hipHostMalloc rows");
  S.rows_cap = c->n_snps;
  return FSCLG_OK;
}

uint32_t* fsclg_slot_row_buffer(fsclg_ctx* c, int slot) {
  if (!c || !c->d_pr0) { set_err(FSCLG_E_STATE, "snps not uploaded"); return nullptr; }
  if (slot < 0 || slot >= NSLOT) { set_err(FSCLG_E_ARG, "slot"); return nullptr; }
  Slot& S = c->slot[slot];
  if (S.users) { set_err(FSCLG_E_STATE, "slot in use by a batch not waited for"); return nullptr; }
  if (hipSetDevice(c->device) != hipSuccess || ensure_row_staging(c, S) != FSCLG_OK) return nullptr;
  // the slot's last upload may still read the buffer
  if (hipEventSynchronize(S.ready) != hipSuccess) { set_err(FSCLG_E_HIP, "hipEventSynchronize"); return nullptr; }
  return S.h_rows;
}

uint32_t* fsclg_row_buffer(fsclg_ctx* c) { return fsclg_slot_row_buffer(c, 0); }

int fsclg_slot_set_rows(fsclg_ctx* c, int slot, const uint32_t* row, const double* chr_null) {
  if (!c || !c->d_pr0) return set_err(FSCLG_E_STATE, "snps not uploaded");
  if (slot < 0 || slot >= NSLOT) return set_err(FSCLG_E_ARG, "slot");
  Slot& S = c->slot[slot];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = ensure_row_staging(c, S))) return r;
  HIPCHK(hipEventSynchronize(S.ready), "hipEventSynchronize");  // the slot's last upload has read the staging
  S.win_valid = false; S.ctab_valid = false;
  if (row) {
    uint32_t mx = 0;
    for (int i = 0; i < c->n_snps; i++) mx = row[i] > mx ? row[i] : mx;  // vectorised validation
    if (mx >= (uint32_t)c->n_rows) return set_err(FSCLG_E_ARG, "row index out of table");
    if (row != S.h_rows) memcpy(S.h_rows, row, sizeof(uint32_t) * c->n_snps);
  }
  if (chr_null) memcpy(S.h_null, chr_null, sizeof(double) * c->n_chr);
  hipLaunchKernelGGL(scatter_rows_kernel<uint32_t>, dim3((c->n_snps + 255) / 256), dim3(64), 0, c->ustream,
                     S.d_pr, row ? S.h_rows : nullptr, c->d_pr0, c->n_snps, S.d_chr_null,
                     chr_null ? S.h_null : nullptr, c->n_chr);
  HIPCHK(hipGetLastError(), "launch scatter_rows_kernel");
  HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");
  return FSCLG_OK;
}

int fsclg_set_rows(fsclg_ctx* c, const uint32_t* row) { return fsclg_slot_set_rows(c, 0, row, nullptr); }

void* fsclg_host_alloc(size_t bytes) {
  void* p = nullptr;
  const hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, HOSTMEM | hipHostMallocPortable);
  if (e != hipSuccess) { set_err(FSCLG_E_HIP, "hipHostMalloc (portable)", e); return nullptr; }
  return p;
}

void fsclg_host_free(void* p) {
  if (p) hipHostFree(p);
}

int fsclg_host_register(void* p, size_t bytes) {
  if (!p || !bytes) return set_err(FSCLG_E_ARG, "host register");
  hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped);
  if (e != hipSuccess) return set_err(FSCLG_E_HIP, "hipHostRegister", e);
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, p, 0);
  if (e != hipSuccess || d != p) {  // the kernels take the host pointer as it is
    hipHostUnregister(p);
    return set_err(e != hipSuccess ? FSCLG_E_HIP : FSCLG_E_STATE, "hipHostGetDevicePointer", e);
  }
  return FSCLG_OK;
}

int fsclg_host_unregister(void* p) {
  if (!p) return FSCLG_OK;
  const hipError_t e = hipHostUnregister(p);
  return e == hipSuccess ? FSCLG_OK : set_err(FSCLG_E_HIP, "hipHostUnregister", e);
}

int fsclg_slot_wait(fsclg_ctx* c, int slot) {
  if (!c) return set_err(FSCLG_E_ARG, "ctx");
  if (slot < 0 || slot >= NSLOT) return set_err(FSCLG_E_ARG, "slot");
  Slot& S = c->slot[slot];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(hipEventSynchronize(S.ready), "hipEventSynchronize");
  return FSCLG_OK;
}

int fsclg_slot_swap(fsclg_ctx* c, int a, int b) {
  if (!c) return set_err(FSCLG_E_ARG, "ctx");
  if (a < 0 || a >= NSLOT || b < 0 || b >= NSLOT) return set_err(FSCLG_E_ARG, "slot");
  if (c->slot[a].users || c->slot[b].users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  if (a != b) std::swap(c->slot[a], c->slot[b]);
  return FSCLG_OK;
}

int fsclg_search_done(fsclg_ctx* c, int batch) {
  if (!c || batch < 0 || batch >= NBATCH) return set_err(FSCLG_E_ARG, "batch");
  Batch& B = c->batch[batch];
  if (!B.pending || B.n_cells == 0) return 1;
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  const hipError_t q = hipEventQuery(B.ev2);
  if (q == hipErrorNotReady) return 0;
  HIPCHK(q, "hipEventQuery");
  return 1;
}

int fsclg_slot_set_rows_host(fsclg_ctx* c, int slot, const uint32_t* row, const double* chr_null) {
  return fsclg_slot_set_rows_packed(c, slot, row, 4, chr_null);
}

int fsclg_slot_set_rows_packed(fsclg_ctx* c, int slot, const void* row, int row_bytes, const double* chr_null) {
  if (!c || !c->d_pr0) return set_err(FSCLG_E_STATE, "snps not uploaded");
  if (!row) return set_err(FSCLG_E_ARG, "rows");
  if (!(row_bytes == 4 || (row_bytes == 2 && c->n_rows <= 0x10000) || (row_bytes == 1 && c->n_rows <= 0x100)))
    return set_err(FSCLG_E_ARG, "row width");
  if (slot < 0 || slot >= NSLOT) return set_err(FSCLG_E_ARG, "slot");
  Slot& S = c->slot[slot];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = ensure_null_staging(c, S))) return r;
  HIPCHK(hipEventSynchronize(S.ready), "hipEventSynchronize");  // the slot's last upload has read h_null
  S.win_valid = false; S.ctab_valid = false;
  if (chr_null) memcpy(S.h_null, chr_null, sizeof(double) * c->n_chr);
  // read straight from the caller's portable pinned rows (one buffer can feed every device)
  const double* cn = chr_null ? S.h_null : nullptr;
  const int per = 64 * (16 / row_bytes);  // sites per block (one wave)
  const dim3 grid((c->n_snps + per - 1) / per);
  if (row_bytes == 1)
    hipLaunchKernelGGL(scatter_rows_kernel<uint8_t>, grid, dim3(64), 0, c->ustream, S.d_pr,
                       static_cast<const uint8_t*>(row), c->d_pr0, c->n_snps, S.d_chr_null, cn, c->n_chr);
  else if (row_bytes == 2)
    hipLaunchKernelGGL(scatter_rows_kernel<uint16_t>, grid, dim3(64), 0, c->ustream, S.d_pr,
                       static_cast<const uint16_t*>(row), c->d_pr0, c->n_snps, S.d_chr_null, cn, c->n_chr);
  else
    hipLaunchKernelGGL(scatter_rows_kernel<uint32_t>, grid, dim3(64), 0, c->ustream, S.d_pr,
                       static_cast<const uint32_t*>(row), c->d_pr0, c->n_snps, S.d_chr_null, cn, c->n_chr);
  HIPCHK(hipGetLastError(), "launch scatter_rows_kernel");
  HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");
  return FSCLG_OK;
}

int fsclg_slot_set_rows_plan(fsclg_ctx* c, int slot, const fsclg_swap_t* ent, const int32_t* grp, int n_grp,
                             const double* chr_null) {
  if (!c || !c->d_pr0) return set_err(FSCLG_E_STATE, "snps not uploaded");
  if (slot < 0 || slot >= NSLOT) return set_err(FSCLG_E_ARG, "slot");
  if (n_grp < 0 || (n_grp > 0 && (!ent || !grp))) return set_err(FSCLG_E_ARG, "plan");
  Slot& S = c->slot[slot];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  // every range inside the sites, kind-0 ranges disjoint, kind 1 alone in its group: a bad plan is
  // an error here, never an out-of-bounds access on the device
  const long long n = c->n_snps;
  int max_rot = 0;
  if (n_grp > 0 && grp[0] != 0) return set_err(FSCLG_E_ARG, "plan groups");
  for (int q = 0; q < n_grp; q++) {
    if (grp[q + 1] <= grp[q]) return set_err(FSCLG_E_ARG, "plan groups");
    for (int e = grp[q]; e < grp[q + 1]; e++) {
      const fsclg_swap_t& x = ent[e];
      const long long d = x.i > x.j ? (long long)x.i - x.j : (long long)x.j - x.i;
      if (x.i < 0 || x.j < 0 || x.len < 0 || x.i + (long long)x.len > n || x.j + (long long)x.len > n)
        return set_err(FSCLG_E_ARG, "plan entry out of range");
      if (x.kind == 0 ? (d < x.len || x.len > 4096) : (x.kind != 1 || d >= x.len || grp[q + 1] - grp[q] != 1))
        return set_err(FSCLG_E_ARG, "plan entry");
      if (x.kind == 1 && x.len + d > max_rot) max_rot = (int)(x.len + d);
    }
  }
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = ensure_null_staging(c, S))) return r;
  if (max_rot > c->plan_tmp_cap) {
    if (c->d_plan_tmp) HIPCHK(hipFree(c->d_plan_tmp), "hipFree");
    c->d_plan_tmp = nullptr; c->plan_tmp_cap = 0;
    HIPCHK(hipMalloc((void**)&c->d_plan_tmp, sizeof(uint32_t) * (size_t)max_rot), "hipMalloc plan");
    c->plan_tmp_cap = max_rot;
  }
  HIPCHK(hipEventSynchronize(S.ready), "hipEventSynchronize");  // the slot's last upload has read h_null
  S.win_valid = false; S.ctab_valid = false;
  if (chr_null) memcpy(S.h_null, chr_null, sizeof(double) * c->n_chr);
  // the uploaded rows (and the null sums), then the groups in order on the same stream
  hipLaunchKernelGGL(scatter_rows_kernel<uint32_t>, dim3((c->n_snps + 255) / 256), dim3(64), 0, c->ustream, S.d_pr,
                     nullptr, c->d_pr0, c->n_snps, S.d_chr_null, chr_null ? S.h_null : nullptr, c->n_chr);
  for (int q = 0; q < n_grp; q++) {
    const fsclg_swap_t& x = ent[grp[q]];
    if (x.kind == 0) {
      hipLaunchKernelGGL(plan_swap_kernel, dim3(grp[q + 1] - grp[q]), dim3(256), 0, c->ustream, S.d_pr, ent, grp[q]);
    } else {
      const int lo = x.i < x.j ? x.i : x.j, d = x.i > x.j ? x.i - x.j : x.j - x.i, R = x.len + d;
      if (d == 0) continue;  // a block swapped with itself
      const dim3 g((unsigned)std::min((R + 255) / 256, 1024));
      hipLaunchKernelGGL(plan_rot_save_kernel, g, dim3(256), 0, c->ustream, S.d_pr, c->d_plan_tmp, lo, R);
      hipLaunchKernelGGL(plan_rot_kernel, g, dim3(256), 0, c->ustream, S.d_pr, c->d_plan_tmp, lo, x.len, d);
    }
  }
  HIPCHK(hipGetLastError(), "launch plan kernels");
  HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");
  return FSCLG_OK;
}

int fsclg_set_chr_null(fsclg_ctx* c, const double* chr_null) {
  if (!c || !c->d_pr0 || !chr_null) return set_err(FSCLG_E_STATE, "snps not uploaded");
  Slot& S = c->slot[0];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = ensure_row_staging(c, S))) return r;
  HIPCHK(hipEventSynchronize(S.ready), "hipEventSynchronize");
  memcpy(S.h_null, chr_null, sizeof(double) * c->n_chr);
  // the null sums only: a one-block scatter over no sites
  hipLaunchKernelGGL(scatter_rows_kernel<uint32_t>, dim3(1), dim3(64), 0, c->ustream, S.d_pr, nullptr, c->d_pr0,
                     0, S.d_chr_null, S.h_null, c->n_chr);
  HIPCHK(hipGetLastError(), "launch scatter_rows_kernel");
  HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");
  return FSCLG_OK;
}

int fsclg_set_alpha_grid(fsclg_ctx* c, const double* coarse, int n_coarse, const double* refine, const int32_t* n_refine) {
  if (!c || !coarse || !refine || !n_refine || n_coarse <= 0 || n_coarse * 2 > MAXWALK) return set_err(FSCLG_E_ARG, "alpha grid");
  for (int i = 0; i <= n_coarse; i++)
    if (n_refine[i] < 0 || n_refine[i] > MAXREF) return set_err(FSCLG_E_ARG, "refine count");
  for (int i = 0; i < n_coarse; i++)  // interval_of relies on x = log(d) + alpha >= LOG_AD_MIN
    if (!(coarse[i] >= LOG_AD_MIN)) return set_err(FSCLG_E_ARG, "alpha below LOG_AD_MIN");
  for (int i = 0; i <= n_coarse; i++)
    for (int r = 0; r < n_refine[i]; r++)
      if (!(refine[i * MAXREF + r] >= LOG_AD_MIN)) return set_err(FSCLG_E_ARG, "alpha below LOG_AD_MIN");
  if (any_pending(c)) return set_err(FSCLG_E_STATE, "search batches in flight");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = upload(&c->d_la_coarse, coarse, (size_t)n_coarse, c->ustream))) return r;
  if ((r = upload(&c->d_la_refine, refine, (size_t)(n_coarse + 1) * MAXREF, c->ustream))) return r;
  if ((r = upload(&c->d_n_refine, n_refine, (size_t)(n_coarse + 1), c->ustream))) return r;
  c->n_coarse = n_coarse;
  c->h_coarse.assign(coarse, coarse + n_coarse);
  c->h_refine.assign(refine, refine + (size_t)(n_coarse + 1) * MAXREF);
  c->h_nref.assign(n_refine, n_refine + n_coarse + 1);
  c->plan_dirty = true;
  return update_dfail(c);
}

// Params::dfail for every alpha of the grid, once both the log table and the grid are set:
// logt3 as a function of |d| (sm-search.c:40-46) is nondecreasing (checked), so the sites of a
// walk are those with logt(|d|) + lalpha <= LOG_AD_MAX, i.e. |d| < dfail
static int update_dfail(fsclg_ctx* c) {
  if (c->h_lt3.empty() || c->h_coarse.empty()) return FSCLG_OK;
  const std::vector<double>& T = c->h_lt3;
  auto lt = [&](uint64_t ad) {
    const uint32_t sh = ad > 0xFFFFFFu ? 16u : (ad > 0xFFFFu ? 8u : 0u);
    return T[(size_t)(ad >> sh) + ((size_t)sh << 13)];
  };
  for (int b = 0; b < 3; b++)  // monotone within each branch's used entries and across branches
    for (int i = (b ? 257 : 1); i < 0x10000; i++)
      if (!(T[(size_t)b * 0x10000 + i - 1] <= T[(size_t)b * 0x10000 + i]))
        return set_err(FSCLG_E_ARG, "log table not monotone");
  if (!(T[0xFFFF] <= T[0x10000 + 256]) || !(T[0x1FFFF] <= T[0x20000 + 256]))
    return set_err(FSCLG_E_ARG, "log table not monotone across branches");
  std::vector<double> las(c->h_coarse);
  las.insert(las.end(), c->h_refine.begin(), c->h_refine.end());
  std::vector<uint32_t> df(las.size());
  for (size_t k = 0; k < las.size(); k++) {
    const double la = las[k];
    auto fails = [&](uint64_t d) { volatile double x = lt(d) + la; return x > LOG_AD_MAX; };
    uint64_t lo = 0, hi = 0xFFFFFFFFull;  // the least failing d in [lo, hi], hi if none below it
    if (!fails(hi)) { df[k] = 0xFFFFFFFFu; continue; }
    while (lo < hi) {
      const uint64_t m = lo + (hi - lo) / 2;
      if (fails(m)) hi = m; else lo = m + 1;
    }
    df[k] = (uint32_t)lo;
  }
  int r = upload(&c->d_dfail, df.data(), df.size(), c->ustream);
  return r ? r : update_dband(c);
}

// Params::dband for every alpha of the grid and every interval threshold: the least |d| with
// fl(logt(|d|) + lalpha) >= thr[j] (the device's own add; logt3 nondecreasing, checked in
// update_dfail), so a site lies in interval j or above iff its |d| reaches dband[alpha][j].
// thr[0] = -inf: 0; thr[n_iv] = +inf: 0xFFFFFFFF (never).  Bands are cut on these.
static int update_dband(fsclg_ctx* c) {
  if (c->h_lt3.empty() || c->h_coarse.empty() || c->h_thr.empty() || c->n_iv <= 0) return FSCLG_OK;
  const std::vector<double>& T = c->h_lt3;
  auto lt = [&](uint64_t ad) {
    const uint32_t sh = ad > 0xFFFFFFu ? 16u : (ad > 0xFFFFu ? 8u : 0u);
    return T[(size_t)(ad >> sh) + ((size_t)sh << 13)];
  };
  std::vector<double> las(c->h_coarse);
  las.insert(las.end(), c->h_refine.begin(), c->h_refine.end());
  const int nd = c->n_iv + 1;
  std::vector<uint32_t> db(las.size() * (size_t)nd);
  for (size_t k = 0; k < las.size(); k++) {
    const double la = las[k];
    for (int j = 0; j < nd; j++) {
      const double th = c->h_thr[j];
      auto reaches = [&](uint64_t d) { volatile double x = lt(d) + la; return x >= th; };
      uint32_t v;
      if (reaches(0)) v = 0;
      else if (!reaches(0xFFFFFFFFull)) v = 0xFFFFFFFFu;
      else {
        uint64_t lo = 0, hi = 0xFFFFFFFFull;  // reaches(lo) false, reaches(hi) true
        while (hi - lo > 1) {
          const uint64_t m = lo + (hi - lo) / 2;
          if (reaches(m)) hi = m; else lo = m;
        }
        v = (uint32_t)hi;
      }
      db[k * nd + j] = v;
    }
  }
  return upload(&c->d_dband, db.data(), db.size(), c->ustream);
}

static int ensure_io(Batch& B, int n) {
  if (n <= B.cap) return FSCLG_OK;
  for (void* p : {(void*)B.p_cells, (void*)B.p_out}) if (p) hipHostFree(p);
  B.p_cells = nullptr; B.p_out = nullptr; B.cap = 0;
  const int cap = n < 1024 ? 1024 : n;
  HIPCHK(hipHostMalloc((void**)&B.p_cells, sizeof(fsclg_cell_t) * cap, HOSTMEM), "hipHostMalloc cells");
  HIPCHK(hipHostMalloc((void**)&B.p_out, sizeof(fsclg_point_t) * cap, HOSTMEM), "hipHostMalloc out");
  B.cap = cap;
  return FSCLG_OK;
}

// add a slot's pending window-kernel time to window_ms (blocks only if it is still running)
static int window_time(fsclg_ctx* c, Slot& S) {
  if (!S.wpend) return FSCLG_OK;
  const double t0 = hprof_on() ? hnow() : 0.0;
  HIPCHK(hipEventSynchronize(S.wev1), "hipEventSynchronize");
  if (hprof_on()) g_hprof[1] += hnow() - t0;
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, S.wev0, S.wev1), "hipEventElapsedTime");
  c->window_ms += ms;
  S.wpend = false;
  return FSCLG_OK;
}

// the null sums of every window of the chromosomes longer than 2*er+1 SNPs, for the slot's
// rows (window_null_kernel on the upload stream, timed apart from the search; the host does
// not wait for it: the slot's batches wait on the GPU, and its time is read later)
typedef cellorder::RangeMemo<fsclg_cell_t, int2> WinMemo;
static int window_ranges(fsclg_ctx* c, int er, const fsclg_cell_t* cells, int n_cells, std::vector<int2>& out,
                         WinMemo& memo);
static int launch_partial_windows(fsclg_ctx* c, Slot& S, int er, const std::vector<int2>& todo);

// window_chunk_kernel's parameters for windows of W sites: emin, the least binade in which a chunk
// of 64 values cannot move the running integer m by 2^52 or more (2^emin >= 64 max |null|), and
// ne binades up to the largest a window's sum can reach (|sum| <= W max |null|); false: use the
// sequential kernel (no finite null value, or binades past the double's integer range)
static bool chunk_params(fsclg_ctx* c, long long W, int& emin, int& ne) {
  double mx = 0.0;
  for (double v : c->h_nullrows) if (std::isfinite(v)) mx = std::max(mx, std::fabs(v));
  if (!(mx > 0.0)) return false;
  int e1 = 0, e2 = 0;
  std::frexp(64.0 * mx, &e1);            // 64 mx < 2^e1
  std::frexp((double)W * mx, &e2);       // W mx < 2^e2: the largest binade is e2 - 1
  emin = e1;
  ne = std::max(1, e2 - e1 + 1);
  return emin + ne - 1 <= 52;
}

// entries per binade of the chunk table: the chunks, then WCG padding entries for a group's reads
static int ctab_stride(const fsclg_ctx* c) { return (c->n_snps + WC - 1) / WC + WCG; }

// window_chunk_kernel's halving search two levels per round trip (FSCLG_WIN_DESC=0: one)
static int win_desc() {
  static const int d = getenv("FSCLG_WIN_DESC") ? atoi(getenv("FSCLG_WIN_DESC")) : 1;
  return d;
}

// the slot's chunk table (after its rows' upload, on the upload stream)
static int ensure_ctab(fsclg_ctx* c, Slot& S, int emin, int ne, long long W) {
  // block levels up to the window's length in chunks (FSCLG_WINDOW_TREE=0: none, one step per chunk)
  static const int tree_on = getenv("FSCLG_WINDOW_TREE") ? atoi(getenv("FSCLG_WINDOW_TREE")) : 1;
  int lmax = 0;
  if (tree_on) while (lmax < CT_LMAX && (2ll << lmax) * WC <= W) lmax++;
  if (S.ctab_valid && S.ctab_emin == emin && S.ctab_ne == ne && S.ctree.lmax == lmax) return FSCLG_OK;
  const int nstride = ctab_stride(c);
  const size_t need = (size_t)nstride * ne;
  if (S.ctab_cap < need) {
    if (S.d_ctab) hipFree(S.d_ctab);
    S.d_ctab = nullptr; S.ctab_cap = 0;
    HIPCHK(hipMalloc((void**)&S.d_ctab, sizeof(double2) * need), "hipMalloc chunk table");
    S.ctab_cap = need;
  }
  S.ctree = CTree{};
  S.ctree.lmax = lmax;
  if (lmax > 0) {
    const int nch = (c->n_snps + WC - 1) / WC;  // chunk indices with a table entry (the last may be NaN)
    size_t tot = 0;
    for (int L = 1; L <= lmax; L++) {
      S.ctree.nb[L] = nch >> L;
      S.ctree.off[L] = (int)tot;
      tot += (size_t)ne * S.ctree.nb[L];
    }
    if (S.ctree_cap < tot) {
      if (S.d_ctree) hipFree(S.d_ctree);
      S.d_ctree = nullptr; S.ctree_cap = 0;
      HIPCHK(hipMalloc((void**)&S.d_ctree, sizeof(double2) * (tot ? tot : 1)), "hipMalloc chunk tree");
      S.ctree_cap = tot;
    }
    S.ctree.p = S.d_ctree;
  }
  // FSCLG_CT_LDS=0: the table without LDS staging (one lane per chunk reading its sites), and every
  // tree level by chunk_tree_kernel
  static const int ct_lds = getenv("FSCLG_CT_LDS") ? atoi(getenv("FSCLG_CT_LDS")) : 1;
  int L1 = 1;  // the first tree level chunk_tree_kernel builds
  if (ct_lds) {
    const int nlev = std::min(CT_SPAN, lmax);
    hipLaunchKernelGGL(chunk_table_lds_kernel, dim3((unsigned)((nstride + 63) / 64)), dim3(256), 0, c->ustream,
                       S.d_pr, c->d_null, c->n_snps, emin, ne, nstride, S.d_ctab, S.ctree, S.d_ctree, nlev);
    L1 = nlev + 1;
  } else {
    const long long nthr = (long long)nstride * ((ne + CT_BG - 1) / CT_BG);
    hipLaunchKernelGGL(chunk_table_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, c->ustream, S.d_pr,
                       c->d_null, c->n_snps, emin, ne, nstride, S.d_ctab);
  }
  HIPCHK(hipGetLastError(), "launch chunk_table_kernel");
  for (int L0 = L1; L0 <= lmax; L0 += CT_SPAN) {  // levels L0 .. L0 + nlev - 1 per launch, from level L0 - 1
    const int nlev = std::min(CT_SPAN, lmax - L0 + 1);
    const int nprev = L0 == 1 ? nstride : S.ctree.nb[L0 - 1];
    const int ngrp = (nprev + 255) / 256;  // four waves of 64 entries per workgroup
    if (ngrp == 0) break;
    hipLaunchKernelGGL(chunk_tree_kernel, dim3((unsigned)(ne * ngrp)), dim3(256), 0, c->ustream, S.d_ctab, nstride,
                       S.ctree, S.d_ctree, L0, nlev, ngrp);
    HIPCHK(hipGetLastError(), "launch chunk_tree_kernel");
  }
  S.ctab_valid = true; S.ctab_emin = emin; S.ctab_ne = ne;
  return FSCLG_OK;
}

static int ensure_windows(fsclg_ctx* c, int slot, int er, const fsclg_cell_t* cells, int n_cells, WinMemo* memo) {
  const long long W = 2ll * er + 1;
  Slot& S = c->slot[slot];
  if (S.win_valid && S.win_er == er && S.win_part) {  // fsclg_slot_windows summed some: anything missing?
    std::vector<int2> need, todo;
    window_ranges(c, er, cells, n_cells, need, *memo);
    size_t d = 0;
    for (int2 x : need) {
      int a = x.x;
      while (d < S.wdone.size() && S.wdone[d].y <= a) d++;
      for (size_t e = d; e < S.wdone.size() && S.wdone[e].x < x.y && a < x.y; e++) {
        if (S.wdone[e].x > a) todo.push_back(make_int2(a, S.wdone[e].x));
        a = std::max(a, S.wdone[e].y);
      }
      if (a < x.y) todo.push_back(make_int2(a, x.y));
    }
    if (todo.empty()) return FSCLG_OK;
    return launch_partial_windows(c, S, er, todo);
  }
  if (S.win_valid && S.win_er == er) return FSCLG_OK;
  // every window start: the chunked kernel (FSCLG_WINDOW_CHUNK=1: the sequential
  // kernel here and the chunked one for partial sets, 0: sequential everywhere)
  const int chunk_mode = getenv("FSCLG_WINDOW_CHUNK") ? atoi(getenv("FSCLG_WINDOW_CHUNK")) : 2;
  int emin = 0, ne = 0;
  const bool chunked = chunk_mode >= 2 && chunk_params(c, W, emin, ne);
  const int per_task = chunked ? WN_WG : WN_WG * WN_PER;
  if (c->wtask_er != er || c->wtask_chunk != (int)chunked) {
    std::vector<int2> tasks;
    for (int ch = 0; ch < c->n_chr; ch++) {
      const long long n = c->h_chr_n[ch];
      if (n <= W) continue;
      const int cnt = (int)(n - W + 1);  // window starts cs .. ce - 2er
      for (int o = 0; o < cnt; o += per_task)
        tasks.push_back(make_int2(c->h_chr_start[ch] + o, std::min(per_task, cnt - o)));
    }
    // every launch reading the task list has completed (no batch runs on a slot being set up;
    // the other slot's window launch ran on this same stream)
    HIPCHK(hipStreamSynchronize(c->ustream), "hipStreamSynchronize");
    c->n_wtasks = (int)tasks.size();
    if (c->n_wtasks > c->wtask_cap) {
      if (c->d_wtasks) hipFree(c->d_wtasks);
      c->d_wtasks = nullptr; c->wtask_cap = 0;
      HIPCHK(hipMalloc((void**)&c->d_wtasks, sizeof(int2) * c->n_wtasks), "hipMalloc window tasks");
      c->wtask_cap = c->n_wtasks;
    }
    if (c->n_wtasks)
      HIPCHK(hipMemcpyAsync(c->d_wtasks, tasks.data(), sizeof(int2) * tasks.size(), hipMemcpyHostToDevice, c->ustream),
             "copy window tasks");
    HIPCHK(hipStreamSynchronize(c->ustream), "hipStreamSynchronize");
    c->wtask_er = er;
    c->wtask_chunk = (int)chunked;
  }
  if (c->n_wtasks) {
    int r;
    if ((r = window_time(c, S))) return r;  // the slot's previous launch (long finished)
    HIPCHK(hipEventRecord(S.wev0, c->ustream), "hipEventRecord");
    if (chunked) {
      if ((r = ensure_ctab(c, S, emin, ne, W))) return r;
      hipLaunchKernelGGL(window_chunk_kernel, dim3(c->n_wtasks), dim3(WN_WG), 0, c->ustream, S.d_pr, c->d_null,
                         c->d_wtasks, (int)W, emin, ne, ctab_stride(c), S.d_ctab, S.d_win_null, S.ctree, win_desc());
    } else {
      hipLaunchKernelGGL((window_null_kernel<WN_PER>), dim3(c->n_wtasks), dim3(WN_WG), 0, c->ustream, S.d_pr,
                         c->d_null, c->d_wtasks, (int)W, S.d_win_null);
    }
    HIPCHK(hipGetLastError(), "launch window_null_kernel");
    HIPCHK(hipEventRecord(S.wev1, c->ustream), "hipEventRecord");
    HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");  // the slot's batches wait for it on the GPU
    S.wpend = true;
  }
  S.win_er = er;
  S.win_valid = true;
  S.win_part = false;
  S.wdone.clear();
  return FSCLG_OK;
}

// the window starts a set of cells can read (one range per cell: a bisection point of the cell
// [start, end] has its nearest SNP in [j(start) - 1, j(end)], search_snppos's j being the least
// index in [1, n) with position >= pos (n if none), and the window start is monotone in the
// nearest SNP), merged, for the chromosomes above 2*er+1 SNPs
static int window_ranges(fsclg_ctx* c, int er, const fsclg_cell_t* cells, int n_cells, std::vector<int2>& out,
                         WinMemo& memo) {
  const long long W = 2ll * er + 1;
  if (!c->sidx_valid) {
    c->site_index.build(c->h_pos.data(), c->h_chr_start.data(), c->h_chr_n.data(), c->n_chr);
    c->sidx_valid = true;
    c->site_epoch++;
  }
  std::vector<int2>& need = c->wr_need;
  memo.ranges(cells, n_cells, (c->site_epoch << 32) | W, need, [&](const fsclg_cell_t& x, int2& rg) {
    const int ch = x.chr;
    if (ch < 0 || ch >= c->n_chr) return false;
    const long long n = c->h_chr_n[ch];
    if (n <= W) return false;
    const int cs = c->h_chr_start[ch], ce = cs + (int)n - 1;
    const int32_t* pos = c->h_pos.data() + cs;
    auto jof = [&](int p) { return c->site_index.find(pos, ch, (int)n, p); };
    const int nlo = std::max(jof(x.start_pos) - 1, 0), nhi = std::min(jof(x.end_pos), (int)n - 1);
    auto wsof = [&](int nl) {
      const int near = cs + nl;
      if (near - er < cs) return cs;
      if (near + er > ce) return std::max(cs, (int)(ce - 2ll * er));
      return near - er;
    };
    rg = make_int2(wsof(nlo), wsof(nhi) + 1);
    return true;
  });
  std::vector<int>& idx = c->wr_idx;
  idx.resize(need.size());
  for (size_t k = 0; k < need.size(); k++) idx[k] = (int)k;
  cellorder::sort_runs(idx, [&need](int a, int b) { return need[a].x < need[b].x; });  // in order already
  out.clear();
  for (int k : idx) {
    const int2& x = need[k];
    if (!out.empty() && x.x <= out.back().y) out.back().y = std::max(out.back().y, x.y);
    else out.push_back(x);
  }
  return FSCLG_OK;
}

// sum the window starts todo (disjoint, sorted) for the slot's rows and add them to wdone
static int launch_partial_windows(fsclg_ctx* c, Slot& S, int er, const std::vector<int2>& todo) {
  // one window per thread (the latency of one sequential chain per window, not four)
  long long blocks = 0;
  for (const int2& x : todo) blocks += (x.y - x.x + WN_WG - 1) / WN_WG;
  if (!blocks) return FSCLG_OK;
  // the slot's previous window launch has read its task list (launches on one stream, in order)
  if (S.wpend) {
    const double t0 = hprof_on() ? hnow() : 0.0;
    HIPCHK(hipEventSynchronize(S.wev1), "hipEventSynchronize");
    if (hprof_on()) g_hprof[1] += hnow() - t0;
  }
  if (S.wtask_cap < blocks) {
    if (S.p_wtasks) hipHostFree(S.p_wtasks);
    S.p_wtasks = nullptr; S.wtask_cap = 0;
    HIPCHK(hipHostMalloc((void**)&S.p_wtasks, sizeof(int2) * blocks, HOSTMEM), "hipHostMalloc window tasks");
    S.wtask_cap = (int)blocks;
  }
  int nt = 0;
  for (const int2& x : todo)
    for (int o = x.x; o < x.y; o += WN_WG) S.p_wtasks[nt++] = make_int2(o, std::min(WN_WG, x.y - o));
  int r;
  if ((r = window_time(c, S))) return r;
  HIPCHK(hipEventRecord(S.wev0, c->ustream), "hipEventRecord");
  // the active cells' windows of one trial (the pruned tail, where each trial waits for them):
  // the chunked kernel, whose chain per window is ~50x shorter (FSCLG_WINDOW_CHUNK=0: sequential)
  const int chunk_mode = getenv("FSCLG_WINDOW_CHUNK") ? atoi(getenv("FSCLG_WINDOW_CHUNK")) : 2;
  int emin = 0, ne = 0;
  if (chunk_mode >= 1 && chunk_params(c, 2ll * er + 1, emin, ne)) {
    if ((r = ensure_ctab(c, S, emin, ne, 2ll * er + 1))) return r;
    hipLaunchKernelGGL(window_chunk_kernel, dim3(nt), dim3(WN_WG), 0, c->ustream, S.d_pr, c->d_null, S.p_wtasks,
                       (int)(2ll * er + 1), emin, ne, ctab_stride(c), S.d_ctab, S.d_win_null, S.ctree, win_desc());
  } else {
    hipLaunchKernelGGL((window_null_kernel<1>), dim3(nt), dim3(WN_WG), 0, c->ustream, S.d_pr, c->d_null, S.p_wtasks,
                       (int)(2ll * er + 1), S.d_win_null);
  }
  HIPCHK(hipGetLastError(), "launch window_null_kernel");
  HIPCHK(hipEventRecord(S.wev1, c->ustream), "hipEventRecord");
  HIPCHK(hipEventRecord(S.ready, c->ustream), "hipEventRecord");  // the slot's batches wait for it on the GPU
  S.wpend = true;
  std::vector<int2> u(S.wdone);
  u.insert(u.end(), todo.begin(), todo.end());
  std::sort(u.begin(), u.end(), [](int2 a, int2 b) { return a.x < b.x; });
  S.wdone.clear();
  for (const int2& x : u) {
    if (!S.wdone.empty() && x.x <= S.wdone.back().y) S.wdone.back().y = std::max(S.wdone.back().y, x.y);
    else S.wdone.push_back(x);
  }
  S.win_er = er; S.win_valid = true; S.win_part = true;
  return FSCLG_OK;
}

// A trial's window null sums for the cells every batch on the slot will evaluate (all of them,
// before the slot's first submit): only those windows when they are few (the pruned tail of a
// long permutation test: a few hundred cells), every window otherwise.  One launch per trial.
static int slot_windows_impl(fsclg_ctx* c, int slot, const fsclg_cell_t* cells, int n_cells, int eval_range);
int fsclg_slot_windows(fsclg_ctx* c, int slot, const fsclg_cell_t* cells, int n_cells, int eval_range) {
  const double t0 = hprof_on() ? hnow() : 0.0;
  const int r = slot_windows_impl(c, slot, cells, n_cells, eval_range);
  if (hprof_on()) g_hprof[0] += hnow() - t0;
  return r;
}
static int slot_windows_impl(fsclg_ctx* c, int slot, const fsclg_cell_t* cells, int n_cells, int eval_range) {
  if (!c || slot < 0 || slot >= NSLOT || (!cells && n_cells) || n_cells < 0 || eval_range < 0)
    return set_err(FSCLG_E_ARG, "slot windows");
  if (!c->d_pr0) return set_err(FSCLG_E_STATE, "snps not uploaded");
  Slot& S = c->slot[slot];
  if (S.users) return set_err(FSCLG_E_STATE, "slot in use by a batch not waited for");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  // the slot's rows unchanged since its sums were made (a trial prepared ahead in a spare slot for
  // a superset of these cells, fsclg_slot_swap): only what is missing
  if (S.win_valid && S.win_er == eval_range) return ensure_windows(c, slot, eval_range, cells, n_cells, &c->wr_memo);
  const long long W = 2ll * eval_range + 1;
  // cost in waves with windows to sum (a wave: 64 threads x WN_PER windows; a block's waves
  // without windows only stage tiles)
  constexpr int WW = 64 * WN_PER;
  long long all = 0;
  for (int ch = 0; ch < c->n_chr; ch++)
    if (c->h_chr_n[ch] > W) all += (c->h_chr_n[ch] - W + 1 + WW - 1) / WW;
  if (!all) return FSCLG_OK;  // no chromosome above the window: the whole-chromosome sums serve
  std::vector<int2> need;
  const double t0 = hprof_on() ? hnow() : 0.0;
  window_ranges(c, eval_range, cells, n_cells, need, c->wr_memo);
  if (hprof_on()) g_hprof[5] += hnow() - t0;
  long long waves = 0;
  for (const int2& x : need) waves += (x.y - x.x + WW - 1) / WW;
  if (2 * waves >= all) {  // most windows: every one, the dense kernel's way
    S.win_valid = false;
    return ensure_windows(c, slot, eval_range, nullptr, 0, nullptr);
  }
  S.wdone.clear();
  S.win_valid = false;
  const double t1 = hprof_on() ? hnow() : 0.0;
  const int r = launch_partial_windows(c, S, eval_range, need);
  if (hprof_on()) g_hprof[6] += hnow() - t1;
  return r;
}


// the best window of K = room / (rows * 32) intervals for a histogram of terms per interval.
// Every row is held: a miss sends the whole wave's gather to the global table, so a row
// prefix (a per-lane miss rate) would miss in nearly every wave, while an interval window
// misses in whole waves (neighbouring sites have nearly equal log distance).
constexpr int BAND_LDS_BYTES = (int)((sizeof(BandLds) + 15) / 16 * 16);
static void choose_window(fsclg_ctx* c, const std::vector<double>& hist) {
  c->c_ivc0 = 0; c->c_civ = 0; c->c_crow = 0; c->c_cover = 0.0;
  c->c_ivc0_b = 0; c->c_civ_b = 0; c->c_cover_b = 0.0;
  const int stat = (int)((sizeof(Smem) + 15) / 16 * 16);
  const int room = LDS_WG - stat - (c->n_iv + 1) * 8 - (c->n_rows + 1) * 8 - (c->lt_hi ? (c->lt_hi - 256) * 8 : 0) -
                   (c->lx_on && FSCLG_LOG_CALC >= 2 ? LX_BYTES + 16 : 0);
  double htot = 0.0;
  for (double h : hist) htot += h;
  if (room < 32 || htot <= 0) return;
  std::vector<double> hpre(c->n_iv + 1, 0.0);
  for (int j = 0; j < c->n_iv; j++) hpre[j + 1] = hpre[j] + hist[j];
  // the best window of K intervals, and its share of the terms
  auto best_iv = [&](int K, int& bj) {
    bj = 0;
    for (int j = 0; j + K <= c->n_iv; j++) if (hpre[j + K] - hpre[j] > hpre[bj + K] - hpre[bj]) bj = j;
    return (hpre[bj + K] - hpre[bj]) / htot;
  };
  // every row of K intervals: a row-prefix cache over more intervals (the most used rows only,
  // the others' lanes from the global table) was measured slower, DESIGN.md §11.5
  const int R = c->n_rows + 1;
  const int K = std::min(c->n_iv, room / (R * 32));
  if (K <= 0) return;
  int bj;
  c->c_cover = best_iv(K, bj);
  c->c_ivc0 = bj; c->c_civ = K; c->c_crow = R;
  // band mode's window: the same choice in the room its BandLds leaves (16 B aligned after the rest)
  const int Kb = std::min(c->n_iv, (room - BAND_LDS_BYTES - 16) / (R * 32));
  if (Kb > 0) { c->c_cover_b = best_iv(Kb, bj); c->c_ivc0_b = bj; c->c_civ_b = Kb; }
}

// Choose the LDS coefficient window: intervals [ivc0, ivc0 + K) x every device row, K * rows
// * 32 bytes beside the static LDS, thresholds and null rows in LDS_WG, maximising the
// expected share of terms it serves (the share of terms in the interval window).  The interval shares come from walks sampled on the host:
// 32 sweep positions spread over the sites, every coarse alpha and the refine grid of the
// first one, every 8th site of each walk, with the device's own log distance.
static void plan_cache(fsclg_ctx* c) {
  c->plan_dirty = false;
  c->c_ivc0 = 0; c->c_civ = 0; c->c_crow = 0; c->c_cover = 0.0;
  c->c_ivc0_b = 0; c->c_civ_b = 0; c->c_cover_b = 0.0;
  if (getenv("FSCLG_NO_WINDOW")) return;  // experiment: every coefficient from the global table
  const int stat = (int)((sizeof(Smem) + 15) / 16 * 16);
  const int room = LDS_WG - stat - (c->n_iv + 1) * 8 - (c->n_rows + 1) * 8 - (c->lt_hi ? (c->lt_hi - 256) * 8 : 0) -
                   (c->lx_on && FSCLG_LOG_CALC >= 2 ? LX_BYTES + 16 : 0);
  if (room < 32 || c->n_iv <= 0 || c->h_pos.empty() || c->h_coarse.empty() || c->h_lt3.empty()) return;
  std::vector<double> hist(c->n_iv, 0.0);
  std::vector<double> las(c->h_coarse);
  for (int k = 0; k < c->h_nref[0]; k++) las.push_back(c->h_refine[k]);
  const double inv = 1.0 / c->step;
  const int S = 32, ST = 8;
  for (int sidx = 0; sidx < S; sidx++) {
    const int i0 = (int)(((long long)sidx * 2 + 1) * c->n_snps / (2 * S));
    int ch = 0;
    while (ch + 1 < c->n_chr && c->h_chr_start[ch + 1] <= i0) ch++;
    const int a = c->h_chr_start[ch], e = a + c->h_chr_n[ch];
    const long long sweep = (long long)c->h_pos[i0] + 1;
    for (double la : las) {
      for (int dir = -1; dir <= 1; dir += 2)
        for (int i = dir < 0 ? i0 : i0 + 1; i >= a && i < e; i += dir * ST) {
          const unsigned long long ad = (unsigned long long)llabs((long long)c->h_pos[i] - sweep);
          const unsigned sh = ad > 0xFFFFFFull ? 16u : (ad > 0xFFFFull ? 8u : 0u);
          const double x = c->h_lt3[(ad >> sh) + ((size_t)sh << 13)] + la;
          if (x > LOG_AD_MAX) break;
          int iv = (int)((x - LOG_AD_MIN) * inv);
          iv = iv < 0 ? 0 : (iv >= c->n_iv ? c->n_iv - 1 : iv);
          hist[iv] += 1.0;
        }
    }
  }
  choose_window(c, hist);
#ifdef FSCLG_IVHIST  // diagnostic builds measure the real histogram in the first launch
  c->hist_pending = true;
#endif
}

// band mode is off by default (-1: the walk-window path with site-major dealing, faster at C4 and C5,
// HISTORY §R6.3); FSCLG_BAND_TH=16 turns it on
static int band_default(const fsclg_ctx* c) { (void)c; return -1; }

static Params make_params(fsclg_ctx* c, Batch& B, int slot, int n, int mode, int eval_range, int bp_resl) {
  const Slot& S = c->slot[slot];
  Params P;
  P.pr = S.d_pr; P.logt3 = c->d_logt; P.coef = c->d_coef; P.nullrow = c->d_null;
  P.thr = c->d_thr; P.n_rows = c->n_rows; P.stride = c->n_rows + 1; P.pstride = P.stride * 16;
  P.inv_step = 1.0 / c->step; P.iv_off = -LOG_AD_MIN * P.inv_step - 1e-9;
  // dynamic LDS: the planned coefficient window, thresholds and null rows
  if (c->plan_dirty) plan_cache(c);
  {
    // band mode (an alternative term order, off by default: HISTORY §R6.1, §R6.3): FSCLG_BAND_TH >= 0
    // turns it on; read per launch, as FSCLG_BAND_NB / FSCLG_BAND_MINP (tests switch them within one
    // process).  Band mode's BandLds sits in the dynamic LDS after the logt copy, so its window is c_civ_b
    const int band_env = getenv("FSCLG_BAND_TH") ? atoi(getenv("FSCLG_BAND_TH")) : -2;
    const int band_th = band_env != -2 ? band_env : band_default(c);
    P.band_th = (c->d_dband && c->d_tpos && c->c_civ_b > 0) ? band_th : -1;
    const int band_nb = getenv("FSCLG_BAND_NB") ? atoi(getenv("FSCLG_BAND_NB")) : NBMAX;
    P.band_nb = band_nb;
    const int band_minp = getenv("FSCLG_BAND_MINP") ? atoi(getenv("FSCLG_BAND_MINP")) : 8;
    P.band_minp = band_minp;
  }
  if (P.band_th >= 0) { P.ivc0 = c->c_ivc0_b; P.n_civ = c->c_civ_b; }
  else { P.ivc0 = c->c_ivc0; P.n_civ = c->c_civ; }
  P.civ_max = std::max(P.n_civ - 1, 0);
  P.n_cache = P.n_civ * P.stride;
  P.off_thr = P.n_cache * 32; P.off_nul = P.off_thr + (c->n_iv + 1) * 8;
  P.off_lt = P.off_nul + (c->n_rows + 1) * 8 - 256 * 8; P.lt_hi = c->lt_hi;  // entry i at off_lt + 8 i
  P.lt_span = c->lt_hi > 256 ? ((uint32_t)c->lt_hi << 16) - 0x1000000u : 0u;  // lt_hi <= 32768
  P.lx = c->d_lx; P.lx_on = FSCLG_LOG_CALC >= 2 ? c->lx_on : 0;  // FSCLG_LOG_CALC=1: set for split launches
  P.off_lx = (P.off_lt + 256 * 8 + (P.lt_hi ? (P.lt_hi - 256) * 8 : 0) + 15) & ~15;
  P.off_bd = ((P.lx_on ? P.off_lx + LX_BYTES : P.off_lt + 256 * 8 + (P.lt_hi ? (P.lt_hi - 256) * 8 : 0)) + 15) & ~15;
  P.chr_start = c->d_chr_start; P.chr_n = c->d_chr_n; P.chr_null = S.d_chr_null; P.win_null = S.d_win_null;
  P.la_coarse = c->d_la_coarse; P.la_refine = c->d_la_refine; P.n_refine = c->d_n_refine;
  P.dfail = c->d_dfail;
  P.dband = c->d_dband; P.nd = c->n_iv + 1; P.tpos = c->d_tpos;
  P.cells = B.p_cells; P.out = B.p_out; P.stats = c->d_stats; P.ctrace = nullptr; P.ivhist = nullptr;
  P.epos = nullptr; P.n_ep = 0; P.ept = nullptr; P.cell_ep = nullptr;
  P.split = 1; P.xacc = nullptr; P.xcnt = nullptr;
  {
    const unsigned long long wait_us =
        getenv("FSCLG_SPLIT_WAIT_US") ? strtoull(getenv("FSCLG_SPLIT_WAIT_US"), nullptr, 10) : 1000000ull;
    const unsigned long long delay_us =
        getenv("FSCLG_TEST_SPLIT_DELAY_US") ? strtoull(getenv("FSCLG_TEST_SPLIT_DELAY_US"), nullptr, 10) : 0ull;
    P.xwait = wait_us * 100ull;  // wall_clock64 runs at 100 MHz
    P.xdelay = delay_us * 100ull;
  }
  P.spec_refine = 0; P.ci_guess = std::min(c->ci_guess, c->n_coarse);
  static const int lookahead = getenv("FSCLG_LOOKAHEAD") ? atoi(getenv("FSCLG_LOOKAHEAD")) : 1;
  P.lookahead = lookahead;
  if (getenv("FSCLG_CELL_TRACE")) {
    if (B.ctrace_cap < n) {
      if (B.p_ctrace) hipHostFree(B.p_ctrace);
      B.p_ctrace = nullptr; B.ctrace_cap = 0;
      if (hipHostMalloc((void**)&B.p_ctrace, sizeof(unsigned long long) * (8 * (size_t)n + 16008), HOSTMEM) == hipSuccess)
        B.ctrace_cap = n;  // + the FSCLG_INST_TRACE event area
    }
    P.ctrace = B.p_ctrace;
  }
  P.n_coarse = c->n_coarse; P.n_iv = c->n_iv; P.step = c->step;
  P.eval_range = eval_range; P.bp_resl = bp_resl; P.n_cells = n; P.mode = mode;
  return P;
}

// split cells' speculative refine walks, off by default since round 4: they cut
// a tail cell's phases from 12 to 9 but measured no shorter job, at one GPU or at 8 (rehearsed),
// and add 8 % to the split segments (§11.3).  FSCLG_SPEC_REFINE=1: on; 2: evaluated but every
// guess taken as missed (the fallback path's test)
static int spec_refine_on() {
  static const int on = getenv("FSCLG_SPEC_REFINE") ? atoi(getenv("FSCLG_SPEC_REFINE")) : 0;
  return on;
}

// the guess for points with no evaluated neighbour: the most frequent coarse alpha index among
// the results so far (a point's lalpha lies within one coarse step of its coarse winner)
static void note_alphas(fsclg_ctx* c, const fsclg_point_t* out, int n) {
  const int nc = std::min(c->n_coarse, 15);
  for (int i = 0; i < n; i++) {
    const double k = floor((out[i].lalpha - LOG_AD_MIN) / 2.4 + 0.5);
    if (k >= 0.0 && k <= (double)nc) c->ci_count[(int)k]++;
  }
  int best = c->ci_guess;
  for (int k = 0; k <= nc; k++) if (c->ci_count[k] > c->ci_count[best]) best = k;
  c->ci_guess = best;
}

// one launch of search_maxpos_kernel with n blocks on the batch's stream (events recorded by the caller)
static int launch_blocks_impl(hipStream_t stream, const Params& P, int n);
static int launch_blocks(hipStream_t stream, const Params& P, int n) {
  const double t0 = hprof_on() ? hnow() : 0.0;
  const int r = launch_blocks_impl(stream, P, n);
  if (hprof_on()) g_hprof[3] += hnow() - t0;
  return r;
}
static int launch_blocks_impl(hipStream_t stream, const Params& P, int n) {
  const int grid = n;
  const int dyn = (P.band_th >= 0 && P.n_civ > 0 && P.split <= 1)
                      ? P.off_bd + BAND_LDS_BYTES
                      : (P.lx_on ? P.off_lx + LX_BYTES : P.off_lt + 256 * 8 + (P.lt_hi ? (P.lt_hi - 256) * 8 : 0));
  const int stat_m = (int)((sizeof(Smem) + 15) / 16 * 16), stat_s = (int)((sizeof(SmemSplit) + 15) / 16 * 16);
  if ((P.split > 1 ? stat_s : stat_m) + dyn <= LDS_WG) {
    static unsigned long long attr_set = 0;  // per device (bit = device id)
    int dev = 0;
    HIPCHK(hipGetDevice(&dev), "hipGetDevice");
    if (dev >= 64 || !(attr_set >> dev & 1ull)) {
      HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&search_maxpos_kernel<true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_WG - stat_m), "hipFuncSetAttribute");
      HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&search_maxpos_kernel<true, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_WG - stat_m), "hipFuncSetAttribute");
      HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&search_maxpos_split_kernel<true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, LDS_WG - stat_s), "hipFuncSetAttribute");
      if (dev < 64) attr_set |= 1ull << dev;
    }
    if (P.split > 1) hipLaunchKernelGGL((search_maxpos_split_kernel<true>), dim3(grid), dim3(WG), dyn, stream, P);
    else if (P.band_th >= 0 && P.n_civ > 0) hipLaunchKernelGGL((search_maxpos_kernel<true, true>), dim3(grid), dim3(WG), dyn, stream, P);
    else hipLaunchKernelGGL((search_maxpos_kernel<true>), dim3(grid), dim3(WG), dyn, stream, P);
  } else
    if (P.split > 1) hipLaunchKernelGGL((search_maxpos_split_kernel<false>), dim3(grid), dim3(WG), 0, stream, P);
    else hipLaunchKernelGGL((search_maxpos_kernel<false>), dim3(grid), dim3(WG), 0, stream, P);
  HIPCHK(hipGetLastError(), "launch search_maxpos_kernel");
  return FSCLG_OK;
}

extern "C++" {
template <typename T>
static int ensure_buf(T** d, int* cap, int n) {
  if (n <= *cap) return FSCLG_OK;
  if (*d) hipFree(*d);
  *d = nullptr; *cap = 0;
  const int k = n < 1024 ? 1024 : n;
  HIPCHK(hipMalloc((void**)d, sizeof(T) * k), "hipMalloc");
  *cap = k;
  return FSCLG_OK;
}
template <typename T>
static int ensure_pinned(T** h, int* cap, int n) {
  if (n <= *cap) return FSCLG_OK;
  if (*h) hipHostFree(*h);
  *h = nullptr; *cap = 0;
  const int k = n < 1024 ? 1024 : n;
  HIPCHK(hipHostMalloc((void**)h, sizeof(T) * k, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc");
  *cap = k;
  return FSCLG_OK;
}
}

// the key of a cell's remembered cost (cell_cost), used only to order a launch longest first:
// distinct below 2^29 bp and 64 chromosomes, and a collision past that misorders, never miscomputes
static unsigned long long cell_key(const fsclg_cell_t& x) {
  return ((unsigned long long)(uint32_t)x.chr << 58) ^ ((unsigned long long)(uint32_t)x.start_pos << 29) ^
         (unsigned long long)(uint32_t)x.end_pos;
}

static int search_submit_impl(fsclg_ctx* c, int batch, int slot, const fsclg_cell_t* cells, int n_cells,
                              int eval_range, int bp_resl);
int fsclg_search_submit(fsclg_ctx* c, int batch, int slot, const fsclg_cell_t* cells, int n_cells, int eval_range,
                        int bp_resl) {
  const double t0 = hprof_on() ? hnow() : 0.0;
  const int r = search_submit_impl(c, batch, slot, cells, n_cells, eval_range, bp_resl);
  if (hprof_on()) g_hprof[2] += hnow() - t0;
  return r;
}
static int search_submit_impl(fsclg_ctx* c, int batch, int slot, const fsclg_cell_t* cells, int n_cells,
                              int eval_range, int bp_resl) {
  if (!c || (!cells && n_cells) || n_cells < 0) return set_err(FSCLG_E_ARG, "cells");
  if (batch < 0 || batch >= NBATCH || slot < 0 || slot >= NSLOT) return set_err(FSCLG_E_ARG, "batch/slot");
  if (!c->d_pr0 || !c->d_coef || !c->d_la_coarse) return set_err(FSCLG_E_STATE, "tables/snps/alpha grid not set");
  Batch& B = c->batch[batch];
  if (B.pending) return set_err(FSCLG_E_STATE, "batch not waited for");
  // host-side shape checks before any launch
  if (eval_range < 0 || bp_resl < 0) return set_err(FSCLG_E_ARG, "eval_range/bp_resl");
  for (int i = 0; i < n_cells; i++) {
    if (cells[i].chr < 0 || cells[i].chr >= c->n_chr) return set_err(FSCLG_E_ARG, "cell chromosome");
    const long long nwin = std::min((long long)c->h_chr_n[cells[i].chr], 2ll * eval_range + 1);
    if (nwin / SEG_SPLIT + 4 > (long long)MAXSEG_W) return set_err(FSCLG_E_UNSUPPORTED, "window above the segment table");
  }
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  B.n_cells = n_cells; B.nu = 0; B.nlaunch = 0; B.slot = slot; B.ivhist = nullptr; B.traced = false;
  B.eval_range = eval_range; B.bp_resl = bp_resl;
  if (n_cells == 0) {
    B.pending = true;
    c->slot[slot].users++;
    return FSCLG_OK;
  }
  {
    const double t0 = hprof_on() ? hnow() : 0.0;
    // the cells' windows (a check against what fsclg_slot_windows summed: each batch remembers its
    // cells' ranges from its previous submit, so this is a merge of two ordered lists)
    if ((r = ensure_windows(c, slot, eval_range, cells, n_cells, &B.wr_memo))) return r;
    if (hprof_on()) g_hprof[4] += hnow() - t0;
  }
  const double t_dd = hprof_on() ? hnow() : 0.0;
  // identical cells are evaluated once (permutation cells are G-aligned, so two points can
  // share one), and so is an endpoint shared by neighbouring cells (scan-chromosome.c:130-134
  // evaluates both ends of every cell): a first launch evaluates the distinct endpoints, the
  // cell launch reads them.  Same inputs, same device arithmetic: identical results.
  // Both by exact comparison in (chromosome, position) order, not hashing (cell_order.h)
  cellorder::dedup_cells(cells, n_cells, B.sidx, B.ucells, B.uidx);
  const int nu = (int)B.ucells.size();
  c->n_dup_cells += (unsigned long long)(n_cells - nu);
  cellorder::dedup_endpoints(B.ucells, B.ekeys, B.sidx, B.epos, B.ucell_ep);
  const int ne = (int)B.epos.size();
  // split cells: a batch of few cells (the permutation pipeline's blocking batch in the
  // pruned tail) gives each cell up to split_max workgroups, within a budget of workgroups.
  // The members of a cell wait for each other, so they must be resident together.  The budget
  // (512, the device's resident slots; 256 where the LDS window pays) and a bulk batch's 128 can
  // together exceed residency when a blocking and a bulk launch run at once: co-residency then
  // rests on the hardware dispatching a launch's workgroups in order (a cell's members are
  // consecutive blocks of one XCD), and where that fails a member's ~1 s wait (PF_SPLIT_TIMEOUT)
  // flags the cell, which is re-run unsplit (n_split_retry; 0 in every committed profile, and
  // test_split_retry_of_a_bulk_batch forces it for a bulk batch)
  int G = 1;
  if (B.split_max > 1) {
    // 512 (round 5): at 8 GPUs C5's tail batches of ~69 cells get 7 members instead of 3 (the rank-0
    // rehearsal 59.7 -> 47.3 s per job, profiles/r05d_c5_ranks); batches of more than 256 cells (every
    // one-GPU job's blocking batches but C5 chr1's) stay unsplit as before
    // 256 where the LDS coefficient window serves much of the terms (C2: 49 %, C3: 35 %), which split
    // launches run without: there 512 cost C2 5 % and C3 9 % per job (HISTORY §R5.13)
    static const int budget_env = getenv("FSCLG_SPLIT_BUDGET") ? atoi(getenv("FSCLG_SPLIT_BUDGET")) : 0;
    const int budget = budget_env > 0 ? budget_env : (c->c_cover >= 0.3 ? 256 : 512);
    // batches 2.. (the permutation pipeline's bulk batches, which run beside a blocking batch that
    // may take the whole budget): a quarter of it, so that only a bulk batch of a few dozen cells
    // is split (the pruned tail at 8 GPUs, a one-chromosome job) and one beside a large unsplit
    // blocking batch (C4's one-GPU tail: 177 bulk cells beside 301) is not
    static const int bulk_budget = getenv("FSCLG_BULK_BUDGET") ? atoi(getenv("FSCLG_BULK_BUDGET")) : 128;
    G = std::min(std::min(B.split_max, MAXSPLIT), (batch >= 2 ? bulk_budget : budget) / std::max(nu, 1));
    if (G < 2) G = 1;
  }
  B.split = G;
  const bool use_ep = G == 1 && !getenv("FSCLG_NO_DEDUP") && (2 * nu - ne) * 8 >= nu;  // saves >= 1/8 of the endpoint work
  // XCD placement of the endpoint launch (two endpoints per block, blocks dealt round-robin
  // over the XCDs): in (chromosome, position) order, the blocks x, x + 8, ... of class x take
  // one consecutive run of endpoints, as the cells below
  if (use_ep && ne >= 16 * 32 && !getenv("FSCLG_NO_XCD")) {
    int nchr = 0, last = -1;
    std::vector<int> loc(ne);
    for (int e = 0; e < ne; e++) loc[e] = e;  // epos is in (chromosome, position) order
    for (int e : loc) if (B.epos[e].x != last) { nchr++; last = B.epos[e].x; }
    if (nchr > 1) {
      const int nb = (ne + 1) / 2;
      std::vector<int> to(ne);
      int k = 0;
      for (int x = 0; x < 8; x++)
        for (int b = x; b < nb; b += 8)
          for (int h = 0; h < 2; h++)
            if (2 * b + h < ne) to[loc[k++]] = 2 * b + h;  // only the last block can hold one
      std::vector<int2> ep2(ne);
      for (int e = 0; e < ne; e++) ep2[to[e]] = B.epos[e];
      B.epos.swap(ep2);
      for (int u = 0; u < nu; u++) B.ucell_ep[u] = make_int2(to[B.ucell_ep[u].x], to[B.ucell_ep[u].y]);
    }
  }
  if (hprof_on()) g_hprof[7] += hnow() - t_dd;
  const double t_or = hprof_on() ? hnow() : 0.0;
  // longest first: each cell's cost in its last launch (permutation trials repeat the cells),
  // else a guess (cells nearer the middle of a chromosome walk further on both sides)
  std::vector<double> cost(nu);
  for (int u = 0; u < nu; u++) {
    const fsclg_cell_t& x = B.ucells[u];
    auto it = c->cell_cost.find(cell_key(x));
    if (it != c->cell_cost.end()) { cost[u] = it->second; continue; }
    const int a = c->h_chr_start[x.chr], nn = c->h_chr_n[x.chr];
    const double lo = c->h_pos[a], hi = c->h_pos[a + nn - 1], span = hi > lo ? hi - lo : 1.0;
    const double m = std::min(std::max(x.start_pos - lo, 0.0), std::max(hi - x.start_pos, 0.0));
    cost[u] = 1e-3 * nn * (1.0 + 2.0 * m / span);
  }
  B.order.resize(nu);
  for (int u = 0; u < nu; u++) B.order[u] = u;
  std::stable_sort(B.order.begin(), B.order.end(), [&](int x, int y) { return cost[x] > cost[y]; });
  // XCD-aware placement (MI355X_MICROARCH.md: blocks are dealt round-robin over the 8 XCDs,
  // so blocks b and b + 8 share one XCD's L2).  With several chromosomes in the launch, each
  // XCD gets a run of consecutive (chromosome, position) cells of 1/8 of the estimated cost,
  // longest first within it: a chromosome's site array then sits in one or two L2s instead of
  // all eight.  Class x takes blocks x, x + 8, ...; a class that runs out leaves idle blocks
  // (chr = -1).  One chromosome: the plain longest-first order.
  int nl = nu;
  {
    int nchr = 0, last = -1;
    std::vector<int> loc(nu);
    for (int u = 0; u < nu; u++) loc[u] = u;  // ucells is in (chromosome, position) order
    for (int u : loc) if (B.ucells[u].chr != last) { nchr++; last = B.ucells[u].chr; }
    if (nchr > 1 && nu >= 8 * 32 && !getenv("FSCLG_NO_XCD")) {
      double tot = 0.0;
      for (int u = 0; u < nu; u++) tot += cost[u];
      std::vector<int> cls(nu);
      double acc = 0.0;
      for (int u : loc) {
        cls[u] = std::min(7, (int)((acc + 0.5 * cost[u]) * 8.0 / tot));
        acc += cost[u];
      }
      std::vector<int> lists[8];
      for (int u : B.order) lists[cls[u]].push_back(u);
      // chromosome-major within a class (longest first within a chromosome): an XCD then works on
      // one of its chromosomes at a time, so its L2 holds one site array instead of its run's
      // three at C5 (measured, DESIGN.md §11.5: -1.1 % per C5 job, -0.6 % per C4 job;
      // FSCLG_XCD_ORDER=0: longest first over the whole class, as before)
      static const int chr_major = getenv("FSCLG_XCD_ORDER") ? atoi(getenv("FSCLG_XCD_ORDER")) : 1;
      if (chr_major)
        for (auto& l : lists)
          std::stable_sort(l.begin(), l.end(), [&](int x, int y) { return B.ucells[x].chr < B.ucells[y].chr; });
      size_t L = 0;
      for (auto& l : lists) L = std::max(L, l.size());
      B.order.assign(8 * L, -1);
      for (size_t j = 0; j < L; j++)
        for (int x = 0; x < 8; x++)
          if (j < lists[x].size()) B.order[8 * j + x] = lists[x][j];
      nl = (int)(8 * L);
    }
  }
  if (hprof_on()) g_hprof[8] += hnow() - t_or;
  if ((r = ensure_io(B, nl))) return r;
  if (use_ep) {
    if ((r = ensure_buf(&B.d_ept, &B.ept_cap, ne))) return r;
    if ((r = ensure_pinned(&B.p_epos, &B.pep_cap, ne))) return r;
    if ((r = ensure_pinned(&B.p_cell_ep, &B.pcep_cap, nl))) return r;
  }
  B.upos.resize(nu);
  for (int k = 0; k < nl; k++) {
    const int u = B.order[k];
    if (u < 0) {  // idle block of the XCD placement
      B.p_cells[k] = fsclg_cell_t{-1, 0, 0};
      if (use_ep) B.p_cell_ep[k] = make_int2(0, 0);
      continue;
    }
    B.p_cells[k] = B.ucells[u];
    if (use_ep) B.p_cell_ep[k] = B.ucell_ep[u];
    B.upos[u] = k;
  }
  if (use_ep) memcpy(B.p_epos, B.epos.data(), sizeof(int2) * ne);
  if (G > 1) {  // the split cells' arrival counters, zeroed before the wait for the slot's rows (the
                // fill then runs while the upload stream still works, off the blocking batch's path)
    const size_t xb = (size_t)nl * 2 * sizeof(XAcc);
    if (B.xacc_cap < xb) {
      if (B.d_xacc) hipFree(B.d_xacc);
      B.d_xacc = nullptr; B.xacc_cap = 0;
      HIPCHK(hipMalloc((void**)&B.d_xacc, xb), "hipMalloc split accumulators");
      B.xacc_cap = xb;
    }
    if ((r = ensure_buf(&B.d_xcnt, &B.xcnt_cap, nl))) return r;
    HIPCHK(hipMemsetAsync(B.d_xcnt, 0, sizeof(unsigned int) * nl, B.stream), "hipMemsetAsync");  // the exchange
                                                                                                  // areas need no zeroing
  }
  // the slot's rows and null sums first
  HIPCHK(hipStreamWaitEvent(B.stream, c->slot[slot].ready, 0), "hipStreamWaitEvent");
  Params P = make_params(c, B, slot, nl, 0, eval_range, bp_resl);
  if (c->hist_pending && P.n_civ > 0) {  // diagnostic builds (FSCLG_IVHIST): per phase key
    const int nh = (c->n_coarse + 2) * c->n_iv;
    if ((r = ensure_buf(&c->d_ivhist, &c->ivhist_n, nh))) return r;
    HIPCHK(hipMemsetAsync(c->d_ivhist, 0, sizeof(unsigned long long) * nh, B.stream), "hipMemset ivhist");
    P.ivhist = c->d_ivhist;
    B.ivhist = c->d_ivhist;
    c->hist_pending = false;
  }
  // the events bracket the kernel launches only (one or two of search_maxpos_kernel)
  HIPCHK(hipEventRecord(B.ev0, B.stream), "hipEventRecord");
  if (use_ep) {
    Params E = P;
    E.mode = 2; E.epos = B.p_epos; E.n_ep = ne; E.ept = B.d_ept; E.n_cells = (ne + 1) / 2; E.ctrace = nullptr;
    if ((r = launch_blocks(B.stream, E, E.n_cells))) return r;
    P.ept = B.d_ept; P.cell_ep = B.p_cell_ep;
    c->n_ep_saved += (unsigned long long)(2 * nu - ne);
  }
  if (G > 1) {
    P.split = G; P.xacc = B.d_xacc; P.xcnt = B.d_xcnt;
    P.spec_refine = spec_refine_on();
    // latency: no LDS coefficient windows (their loads, repeated by every member for every
    // phase, cost more than the global gathers of a lightly loaded device)
    P.ivc0 = 0; P.n_civ = 0; P.civ_max = 0; P.n_cache = 0;
    P.off_thr = 0; P.off_nul = (c->n_iv + 1) * 8;
    P.off_lt = P.off_nul + (c->n_rows + 1) * 8 - 256 * 8;
    P.off_lx = (P.off_lt + 256 * 8 + (P.lt_hi ? (P.lt_hi - 256) * 8 : 0) + 15) & ~15;
    P.lx_on = FSCLG_LOG_CALC >= 1 ? c->lx_on : 0;
  }
  if ((r = launch_blocks(B.stream, P, G > 1 ? (nl + 7) / 8 * 8 * G : nl))) return r;
  HIPCHK(hipEventRecord(B.ev1, B.stream), "hipEventRecord");
  HIPCHK(hipEventRecord(B.ev2, B.stream), "hipEventRecord");
  B.traced = P.ctrace != nullptr;
  B.trace_n = nl;
  B.nu = nl;
  B.nlaunch = use_ep ? 2 : 1;
  B.pending = true;
  c->slot[slot].users++;
  return FSCLG_OK;
}

int fsclg_search_wait(fsclg_ctx* c, int batch, fsclg_point_t* out) {
  if (!c || batch < 0 || batch >= NBATCH) return set_err(FSCLG_E_ARG, "batch");
  Batch& B = c->batch[batch];
  if (!B.pending) return set_err(FSCLG_E_STATE, "batch not submitted");
  if (!out && B.n_cells) return set_err(FSCLG_E_ARG, "out");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  B.pending = false;
  c->slot[B.slot].users--;
  if (B.n_cells == 0) return FSCLG_OK;
  const int nu = B.nu;
  // the batch's own completion (its stream may hold later batches): the D2H after ev1
  HIPCHK(hipEventSynchronize(B.ev2), "hipEventSynchronize");
  float ms = 0.f, t0 = 0.f, t1 = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, B.ev0, B.ev1), "hipEventElapsedTime");
  HIPCHK(hipEventElapsedTime(&t0, c->ev_ref, B.ev0), "hipEventElapsedTime");
  HIPCHK(hipEventElapsedTime(&t1, c->ev_ref, B.ev1), "hipEventElapsedTime");
  c->kernel_ms += ms;
  c->launches += (unsigned long long)B.nlaunch;
  c->busy.emplace_back((double)t0, (double)t1);
  if (B.ivhist) {  // re-plan the LDS window from the measured histogram
    const int nkey = c->n_coarse + 2;
    std::vector<unsigned long long> hk((size_t)nkey * c->n_iv), h(c->n_iv, 0);
    HIPCHK(hipMemcpy(hk.data(), B.ivhist, sizeof(unsigned long long) * hk.size(), hipMemcpyDeviceToHost), "copy ivhist");
    for (int k = 0; k < nkey; k++)
      for (int j = 0; j < c->n_iv; j++) h[j] += hk[(size_t)k * c->n_iv + j];
    choose_window(c, std::vector<double>(h.begin(), h.end()));
    B.ivhist = nullptr;
  }
  if (B.traced) {  // development aid: append [n, then n x (start, end, cu, terms, 4 phase times)] to the file
    std::vector<unsigned long long> h((size_t)8 * nu);
    memcpy(h.data(), B.p_ctrace, sizeof(unsigned long long) * h.size());
    if (const char* ie = getenv("FSCLG_INST_TRACE_FILE")) {  // cell 0's events: [count, 4 x count]
      const unsigned long long* q = B.p_ctrace + 8 * (size_t)B.trace_n;
      if (FILE* f = fopen(ie, "ab")) {
        fwrite(q, sizeof(unsigned long long), 1 + 4 * (size_t)std::min(q[0], 4000ull), f);
        fclose(f);
      }
      memset(B.p_ctrace + 8 * (size_t)B.trace_n, 0, sizeof(unsigned long long) * 16008);
    }
    if (FILE* f = fopen(getenv("FSCLG_CELL_TRACE"), "ab")) {  // header: n | batch << 40 | split << 48
      const unsigned long long nn = (unsigned long long)nu | ((unsigned long long)batch << 40) |
                                    ((unsigned long long)B.split << 48);
      fwrite(&nn, sizeof nn, 1, f);
      fwrite(h.data(), sizeof(unsigned long long), h.size(), f);
      fclose(f);
    }
  }
  for (int k = 0; k < nu; k++)
    if (B.p_cells[k].chr >= 0) c->cell_cost[cell_key(B.p_cells[k])] = B.p_out[k].cost;
  for (int i = 0; i < B.n_cells; i++) out[i] = B.p_out[B.upos[B.uidx[i]]];
  // a split cell whose members were not all resident at once (a member waited > ~1 s: a busy
  // or shared device) has no result: the launch is run again with one workgroup per cell,
  // which needs no co-residency and gives the same results
  bool retry = false;
  for (int i = 0; i < B.n_cells && !retry; i++) retry = (out[i].flags & PF_SPLIT_TIMEOUT) && B.split > 1;
  {  // FSCLG_FORCE_SPLIT_RETRY=n (tests): treat split launches as timed out until n retries were
     // counted since the last fsclg_reset_stats; FSCLG_FORCE_SPLIT_RETRY_MINBATCH=b: only those of
     // batches >= b (2: the permutation pipeline's bulk batches)
    const char* fe = getenv("FSCLG_FORCE_SPLIT_RETRY");
    const char* fb = getenv("FSCLG_FORCE_SPLIT_RETRY_MINBATCH");
    if (!retry && B.split > 1 && fe && c->n_split_retry < (unsigned long long)atoll(fe) && (!fb || batch >= atoi(fb)))
      retry = true;
  }
  if (retry) {
    std::vector<fsclg_cell_t> cells(B.n_cells);
    for (int i = 0; i < B.n_cells; i++) cells[i] = B.ucells[B.uidx[i]];
    const int saved = B.split_max;
    c->n_split_retry++;
    B.split_max = 1;
    int r = fsclg_search_submit(c, batch, B.slot, cells.data(), B.n_cells, B.eval_range, B.bp_resl);
    B.split_max = saved;
    if (r) return r;
    return fsclg_search_wait(c, batch, out);
  }
  note_alphas(c, out, B.n_cells);
  for (int i = 0; i < B.n_cells; i++)
    if (out[i].flags)
      return set_err(out[i].flags & PF_UNSUPPORTED ? FSCLG_E_UNSUPPORTED : FSCLG_E_KERNEL,
                     out[i].flags & PF_SPLIT_TIMEOUT ? "device flag: a split cell's members were not resident together"
                                                     : "device flag");
  return FSCLG_OK;
}

int fsclg_set_batch_split(fsclg_ctx* c, int batch, int max_members) {
  if (!c || batch < 0 || batch >= NBATCH || max_members < 1) return set_err(FSCLG_E_ARG, "batch split");
  c->batch[batch].split_max = std::min(max_members, MAXSPLIT);
  return FSCLG_OK;
}

int fsclg_search_maxpos(fsclg_ctx* c, const fsclg_cell_t* cells, int n_cells, int eval_range, int bp_resl,
                        fsclg_point_t* out) {
  if (!c || (!cells && n_cells) || (!out && n_cells) || n_cells < 0) return set_err(FSCLG_E_ARG, "cells");
  if (!c->d_pr0 || !c->d_coef || !c->d_la_coarse) return set_err(FSCLG_E_STATE, "tables/snps/alpha grid not set");
  if (n_cells == 0) return FSCLG_OK;
  int r = fsclg_search_submit(c, 0, 0, cells, n_cells, eval_range, bp_resl);
  if (r) return r;
  return fsclg_search_wait(c, 0, out);
}

int fsclg_search_points(fsclg_ctx* c, fsclg_point_t* pts, int n_pts) {
  if (!c || (!pts && n_pts) || n_pts < 0) return set_err(FSCLG_E_ARG, "points");
  if (!c->d_pr0 || !c->d_coef || !c->d_la_coarse) return set_err(FSCLG_E_STATE, "tables/snps/alpha grid not set");
  if (n_pts == 0) return FSCLG_OK;
  Batch& B = c->batch[0];
  if (B.pending) return set_err(FSCLG_E_STATE, "batch 0 not waited for");
  for (int i = 0; i < n_pts; i++) {
    const fsclg_point_t& p = pts[i];
    if (p.window_start < 0 || p.window_end >= c->n_snps || p.window_start > p.window_end ||
        p.nearest_snp < p.window_start || p.nearest_snp > p.window_end)
      return set_err(FSCLG_E_ARG, "point window");
    if ((p.window_end - p.window_start + 1) / SEG_SPLIT + 4 > MAXSEG_W) return set_err(FSCLG_E_UNSUPPORTED, "window above the segment table");
  }
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  int r;
  if ((r = ensure_io(B, n_pts))) return r;
  HIPCHK(hipStreamWaitEvent(B.stream, c->slot[0].ready, 0), "hipStreamWaitEvent");
  memcpy(B.p_out, pts, sizeof(fsclg_point_t) * n_pts);  // read and written in place by the kernel
  Params P = make_params(c, B, 0, n_pts, 1, 0, 0);
  // latency (the reference's scan loop calls search_maxalpha once per point): a few points get
  // up to FSCLG_POINTS_SPLIT workgroups each (default 8), which share every walk's segments as
  // a split cell's members do
  static const int psplit = getenv("FSCLG_POINTS_SPLIT") ? atoi(getenv("FSCLG_POINTS_SPLIT")) : 8;
  int G = std::min(std::min(psplit, MAXSPLIT), 256 / n_pts);
  if (G < 2) G = 1;
  if (G > 1) {
    const int nl = (n_pts + 7) / 8 * 8;
    const size_t xb = (size_t)nl * 2 * sizeof(XAcc);
    if (B.xacc_cap < xb) {
      if (B.d_xacc) hipFree(B.d_xacc);
      B.d_xacc = nullptr; B.xacc_cap = 0;
      HIPCHK(hipMalloc((void**)&B.d_xacc, xb), "hipMalloc split accumulators");
      B.xacc_cap = xb;
    }
    if ((r = ensure_buf(&B.d_xcnt, &B.xcnt_cap, nl))) return r;
    HIPCHK(hipMemsetAsync(B.d_xcnt, 0, sizeof(unsigned int) * nl, B.stream), "hipMemsetAsync");
    P.split = G; P.xacc = B.d_xacc; P.xcnt = B.d_xcnt;
    P.spec_refine = spec_refine_on();
    P.ivc0 = 0; P.n_civ = 0; P.civ_max = 0; P.n_cache = 0;  // as a split batch: no LDS coefficient windows
    P.off_thr = 0; P.off_nul = (c->n_iv + 1) * 8;
    P.off_lt = P.off_nul + (c->n_rows + 1) * 8 - 256 * 8;
    P.off_lx = (P.off_lt + 256 * 8 + (P.lt_hi ? (P.lt_hi - 256) * 8 : 0) + 15) & ~15;
  }
  HIPCHK(hipEventRecord(B.ev0, B.stream), "hipEventRecord");
  if ((r = launch_blocks(B.stream, P, G > 1 ? (n_pts + 7) / 8 * 8 * G : n_pts))) return r;
  HIPCHK(hipEventRecord(B.ev1, B.stream), "hipEventRecord");
  HIPCHK(hipEventSynchronize(B.ev1), "hipEventSynchronize");
  memcpy(pts, B.p_out, sizeof(fsclg_point_t) * n_pts);
  note_alphas(c, pts, n_pts);
  for (int i = 0; i < n_pts; i++)
    if (pts[i].flags & (PF_UNSUPPORTED | PF_SPLIT_TIMEOUT))
      return set_err(pts[i].flags & PF_UNSUPPORTED ? FSCLG_E_UNSUPPORTED : FSCLG_E_KERNEL,
                     pts[i].flags & PF_SPLIT_TIMEOUT ? "device flag: a point's members were not resident together"
                                                     : "device flag");
  float ms = 0.f, t0 = 0.f, t1 = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, B.ev0, B.ev1), "hipEventElapsedTime");
  HIPCHK(hipEventElapsedTime(&t0, c->ev_ref, B.ev0), "hipEventElapsedTime");
  HIPCHK(hipEventElapsedTime(&t1, c->ev_ref, B.ev1), "hipEventElapsedTime");
  c->kernel_ms += ms;
  c->launches++;
  c->busy.emplace_back((double)t0, (double)t1);
  return FSCLG_OK;
}

int fsclg_interval_thresholds(double log_ad_step, int n_iv, double* thr) {
  if (!thr || n_iv <= 0 || !(log_ad_step > 0)) return set_err(FSCLG_E_ARG, "thresholds");
  thr[0] = 0.0;
  for (int j = 1; j <= n_iv; j++) thr[j] = interval_threshold(j, log_ad_step);
  return FSCLG_OK;
}

int fsclg_get_stats(fsclg_ctx* c, fsclg_stats_t* st) {
  if (!c || !st) return set_err(FSCLG_E_ARG, "stats");
  unsigned long long h[8];
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(hipMemcpy(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost), "copy stats");
#ifdef FSCLG_TRIP_STAMPS
  {
    unsigned long long t[16];
    HIPCHK(hipMemcpy(t, c->d_stats + 8, sizeof t, hipMemcpyDeviceToHost), "copy stamps");
    const double n = t[0] ? (double)t[0] : 1.0;
    fprintf(stderr, "[trip stamps] trips %llu  cycles/trip: nx+|d| %.0f  log+interval %.0f  coef+poly %.0f  sums %.0f\n"
                    "  coef path trips LDS %llu global %llu per-lane %llu; coef+poly cycles/trip %.0f / %.0f / %.0f\n"
                    "  log path trips LDS-far %llu mid %llu per-lane %llu; log+interval cycles/trip mid %.0f far %.0f\n",
            t[0], t[1] / n, t[2] / n, t[3] / n, t[4] / n, t[5], t[6], t[7], t[8] / (t[5] ? (double)t[5] : 1.0),
            t[9] / (t[6] ? (double)t[6] : 1.0), t[10] / (t[7] ? (double)t[7] : 1.0), t[11], t[12], t[13],
            t[14] / (t[12] ? (double)t[12] : 1.0), t[15] / (t[11] ? (double)t[11] : 1.0));
  }
#endif
  memset(st, 0, sizeof *st);
  st->n_terms = h[0]; st->n_null = h[1]; st->n_walks = h[2]; st->n_maxalpha = h[3];
  st->n_unsafe = h[4]; st->n_slow = h[5]; st->n_ties = h[6]; st->n_cells = h[7];
  for (int k = 0; k < NSLOT; k++) window_time(c, c->slot[k]);
  st->kernel_ms = c->kernel_ms; st->n_launches = c->launches; st->window_ms = c->window_ms;
  st->n_dup_cells = c->n_dup_cells; st->n_ep_saved = c->n_ep_saved;
  st->n_split_retry = c->n_split_retry;
  {  // union of the batches' kernel intervals
    std::vector<std::pair<double, double>> iv(c->busy);
    std::sort(iv.begin(), iv.end());
    double busy = 0.0, a = 0.0, b = -1.0;
    for (const auto& x : iv) {
      if (x.first > b) { if (b > a) busy += b - a; a = x.first; b = x.second; }
      else b = std::max(b, x.second);
    }
    if (b > a) busy += b - a;
    st->busy_ms = busy;
  }
  if (c->plan_dirty) plan_cache(c);
  if (band_default(c) >= 0) { st->cache_iv0 = c->c_ivc0_b; st->cache_n_iv = c->c_civ_b; st->cache_cover = c->c_cover_b; }
  else { st->cache_iv0 = c->c_ivc0; st->cache_n_iv = c->c_civ; st->cache_cover = c->c_cover; }
  st->cache_n_rows = c->c_crow;
  return FSCLG_OK;
}

int fsclg_reset_stats(fsclg_ctx* c) {
  if (!c) return set_err(FSCLG_E_ARG, "stats");
  HIPCHK(hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(hipMemset(c->d_stats, 0, sizeof(unsigned long long) * 24), "hipMemset");
  for (int k = 0; k < NSLOT; k++) window_time(c, c->slot[k]);  // pending times belong before the reset
  c->kernel_ms = 0.0; c->launches = 0; c->window_ms = 0.0; c->n_dup_cells = 0; c->n_ep_saved = 0; c->n_split_retry = 0;
  c->busy.clear();
  return FSCLG_OK;
}

}  // extern "C"
