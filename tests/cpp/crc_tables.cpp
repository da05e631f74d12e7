// Dumps, as JSON, the CRC-32 and GF(2^8) tables the engine uses, for
// tests/test_nrs_apache.py (GF tables vs the reference's GF256 literals) and
// tests/test_crc_tables.py to compare with the reference's own tables
// (tests/golden/crc32_tables.json <- hadoop-common's
// crc32_zlib_polynomial_tables.h): the slicing tables as laid out in the
// window kernels' LDS image (every bank-private copy checked equal), the
// image's zero-append tables, and T8_4..T8_7 computed by the engine's Z_n
// operator (a byte followed by j zero bytes = Z_j applied to T8_0).
// Host code only; built with hipcc for the HIP headers hrs_crc.hpp includes.
#include <cstdio>
#include <vector>

#include "../../lambdafs_amd/csrc/gf256.hpp"
#include "../../lambdafs_amd/csrc/hrs_crc.hpp"

namespace cr = hrs::crc;

static void dump(const char* name, const uint32_t* v, int n, bool last = false) {
  std::printf("\"%s\": [", name);
  for (int i = 0; i < n; ++i) std::printf("%s%u", i ? ", " : "", v[i]);
  std::printf("]%s\n", last ? "" : ",");
}

int main() {
  const std::vector<uint32_t> img = hrs::crc_window_image(cr::kPieceBytes, cr::kChunkBytes);
  std::printf("{\n");
  for (int j = 0; j < 4; ++j) {
    uint32_t t[256];
    for (int v = 0; v < 256; ++v) {
      t[v] = img[hrs::crc_slice_word(j, v, 0)];
      for (int r = 1; r < hrs::kCrcRep; ++r)
        if (img[hrs::crc_slice_word(j, v, r)] != t[v]) {
          std::fprintf(stderr, "slice table %d entry %d copy %d differs\n", j, v, r);
          return 1;
        }
    }
    char name[32];
    std::snprintf(name, sizeof name, "lds_slice_T8_%d", j);
    dump(name, t, 256);
  }
  const cr::ByteTable t0 = cr::make_t0();
  for (int j = 4; j < 8; ++j) {  // via the engine's zero-append operator
    const cr::Mat z = cr::zeros(j);
    uint32_t t[256];
    for (int v = 0; v < 256; ++v) t[v] = cr::apply(z, t0.t[v]);
    char name[32];
    std::snprintf(name, sizeof name, "zeros_T8_%d", j);
    dump(name, t, 256);
  }
  {  // the engine's GF(2^8) tables (gf256.hpp: host matrices, byte-granular kernels)
    const hrs::gf::Tables g = hrs::gf::make_tables();
    uint32_t e[512], l[256];
    for (int i = 0; i < 512; ++i) e[i] = g.exp[i];
    for (int i = 0; i < 256; ++i) l[i] = g.log[i];
    dump("gf_exp", e, 512);
    dump("gf_log", l, 256);
  }
  dump("lds_z_chunk", &img[hrs::kCrcSliceWords], 1024);
  dump("lds_z_tree", &img[hrs::kCrcSliceWords + 1024], 6 * 1024, true);
  std::printf("}\n");
  return 0;
}
