// Host-side checks of the index math the kernels rely on, built with AddressSanitizer and
// UndefinedBehaviorSanitizer on the host code only (scripts/sanitize_host.sh; GPU sanitizers are not
// available on this pool). A wrong mapping here is a silent wrong result or an out-of-bounds access
// on the GPU, so each property is checked exhaustively over the shapes that matter:
//
//  * tile_order / xcd_remap (fa_common.h): every causal / non-causal FA2 grid maps block ids to
//    (batch*head, tile level) BIJECTIVELY, for every head-group size the host can pick;
//  * swz / lds_off: the XOR-swizzled LDS images keep every 16-B chunk of a row inside the row and
//    the row-fragment (ds_read_b128) and transposed (ds_read_b64_tr_b16) reads bank-conflict free
//    for every row width the kernels instantiate (64, 128, 192, 256 B);
//  * stream_k_mode / macro_tile_area (tensile_names.h): the Tensile name parsing behind the
//    concurrency-safe GEMM selection.
#include <cstdio>
#include <set>
#include <vector>

#include "cs336/tensile_names.h"
#include "fa_common.h"

using namespace cs336;
using namespace cs336::fa;

static int failures = 0;
#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      ++failures;                             \
      std::fprintf(stderr, "FAIL: " __VA_ARGS__); \
      std::fprintf(stderr, "\n");             \
    }                                         \
  } while (0)

static void check_tile_order() {
  const int nbhs[] = {1, 3, 6, 8, 16, 24, 64, 600, 384};
  const int nts[] = {1, 2, 4, 5, 8, 32, 128};
  const int grps[] = {1, 2, 3, 8, 1 << 20};
  long checked = 0;
  for (int nbh : nbhs)
    for (int nt : nts)
      for (int order = 0; order <= 2; ++order)
        for (int grp : grps) {
          std::vector<char> seen((size_t)nbh * nt, 0);
          for (int bid = 0; bid < nbh * nt; ++bid) {
            int bh = -1, lvl = -1;
            tile_order(bid, nbh, nt, order, grp, bh, lvl);
            CHECK(bh >= 0 && bh < nbh && lvl >= 0 && lvl < nt, "tile_order out of range nbh=%d nt=%d order=%d grp=%d bid=%d -> (%d,%d)",
                  nbh, nt, order, grp, bid, bh, lvl);
            if (bh < 0 || bh >= nbh || lvl < 0 || lvl >= nt) continue;
            char& s = seen[(size_t)bh * nt + lvl];
            CHECK(!s, "tile_order not injective nbh=%d nt=%d order=%d grp=%d (%d,%d)", nbh, nt, order, grp, bh, lvl);
            s = 1;
            ++checked;
          }
        }
  for (int total : {1, 7, 8, 9, 255, 256, 257, 2400, 4801}) {
    std::set<int> ids;
    for (int b = 0; b < total; ++b) ids.insert(xcd_remap(b, total));
    CHECK((int)ids.size() == total && *ids.begin() == 0 && *ids.rbegin() == total - 1, "xcd_remap not a permutation of %d", total);
  }
  std::printf("tile_order: %ld block ids checked\n", checked);
}

template <int RB>
static void check_swizzle() {
  constexpr int CPR = RB / 16;
  // chunks stay in their row and the map is a permutation of the row's chunks
  for (int r = 0; r < 256; ++r) {
    std::set<int> phys;
    for (int c = 0; c < CPR; ++c) {
      const int off = lds_off<RB>(r, c);
      CHECK(off >= r * RB && off < (r + 1) * RB && off % 16 == 0, "RB=%d row %d chunk %d leaves its row", RB, r, c);
      phys.insert(off);
    }
    CHECK((int)phys.size() == CPR, "RB=%d row %d: swizzle is not a permutation", RB, r);
  }
  // ds_read_b128 row fragments: 4 groups of 16 lanes, lane -> row r0 + (lane & 31), chunk 2ks + (lane >> 5)
  const int g128[2][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                           {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31}};
  int worst = 0;
  for (int r0 = 0; r0 < 128; r0 += 32)
    for (int ks = 0; 2 * ks + 1 < CPR; ++ks)
      for (int hi = 0; hi < 2; ++hi)
        for (const auto& g : g128) {
          int banks[64] = {0};
          for (int l : g) {
            const int lane = l + 32 * hi;
            const int a = lds_off<RB>(r0 + (lane & 31), 2 * ks + (lane >> 5));
            for (int w = 0; w < 4; ++w) ++banks[(a / 4 + w) % 64];
          }
          for (int b : banks) worst = b > worst ? b : worst;
        }
  CHECK(worst <= 1, "RB=%d ds_read_b128 row fragments: %d-way bank conflict", RB, worst);
  // ds_read_b64_tr_b16 (lds_tr_frag): one instruction = 32 lanes, rows row0+16s+4h+(i>>2) (+8 for the
  // second read), chunk dt*4 + gq*2 + ((i&3)>>1), 8 B at (i&1)*8
  int worst_tr = 0;
  const int ndt = RB / 64;  // 32-wide d tiles
  for (int row0 = 0; row0 < 128; row0 += 32)
    for (int s = 0; s < 2; ++s)
      for (int dt = 0; dt < ndt; ++dt)
        for (int h = 0; h < 2; ++h)
          for (int second = 0; second < 2; ++second) {
            int banks[64] = {0};
            for (int lane = 32 * h; lane < 32 * h + 32; ++lane) {
              const int i = lane & 15, gq = (lane >> 4) & 1;
              const int c = dt * 4 + gq * 2 + ((i & 3) >> 1);
              const int r = row0 + 16 * s + 4 * h + (i >> 2) + 8 * second;
              const int a = lds_off<RB>(r, c) + (i & 1) * 8;
              for (int w = 0; w < 2; ++w) ++banks[(a / 4 + w) % 64];
            }
            for (int b : banks) worst_tr = b > worst_tr ? b : worst_tr;
          }
  CHECK(worst_tr <= 1, "RB=%d ds_read_b64_tr_b16: %d-way bank conflict", RB, worst_tr);
  std::printf("swizzle RB=%d: row-fragment reads %d-way, transposed reads %d-way\n", RB, worst, worst_tr);
}

static void check_names() {
  CHECK(stream_k_mode("Cijk_Alik_Bljk_BBS_MT160x256x64_SS1_SK3_SKFTR0_SKXCCM8_TLDS1_WG32_8_1") == 3, "SK3");
  CHECK(stream_k_mode("Cijk_Ailk_Bjlk_BSS_MT256x256x64_SK0_SKXCCM0_WG32_8_1") == 0, "SK0");
  CHECK(stream_k_mode("Cijk_Ailk_Bjlk_MT128x128x64_SKXCCM8_WG32") == 0, "no SK token");
  CHECK(stream_k_mode("x_SK12") == 12, "trailing SK12");
  CHECK(stream_k_mode("") == 0 && stream_k_mode("_SK") == 0 && stream_k_mode("_SK_") == 0, "degenerate names");
  CHECK(macro_tile_area("Cijk_MT160x256x64_MI16") == 160 * 256, "MT160x256");
  CHECK(macro_tile_area("Cijk_noMT") == 0 && macro_tile_area("_MTx") == 0, "no MT");
}

// the dK/dV kernel's row-constant staging: row_perm is a bijection on each 64-row tile that puts
// accumulator register reg of lane-half h (32-row group t) at 32t + 16h + reg, and the LDS-DMA
// source chunks land the same rows in the same places
static void check_row_perm() {
  std::set<int> seen;
  for (int r = 0; r < 64; ++r) {
    CHECK(row_perm(r) >= 0 && row_perm(r) < 64, "row_perm(%d) out of range", r);
    seen.insert(row_perm(r));
  }
  CHECK(seen.size() == 64, "row_perm is not a bijection on 0..63");
  for (int t = 0; t < 2; ++t)
    for (int h = 0; h < 2; ++h)
      for (int reg = 0; reg < 16; ++reg)
        CHECK(row_perm(32 * t + acc_row(reg, h)) == 32 * t + 16 * h + reg, "row_perm t %d h %d reg %d", t, h, reg);
  for (int c = 0; c < 16; ++c)
    for (int u = 0; u < 4; ++u)
      CHECK(row_perm(4 * row_perm_src_chunk(c) + u) == 4 * c + u, "DMA chunk %d element %d", c, u);
}

int main() {
  check_row_perm();
  check_tile_order();
  check_swizzle<64>();
  check_swizzle<128>();
  check_swizzle<192>();
  check_swizzle<256>();
  check_names();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host checks passed\n");
  return 0;
}
