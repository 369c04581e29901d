// Host build of pinot_amd/csrc/codec.h for the CPU tests (tests/test_codec.py): the same decoder source the GPU
// chunk decode runs, exercised against zlib / libzstd outputs.
#include <stdint.h>
#include <vector>

#include "../../pinot_amd/csrc/codec.h"

extern "C" int phip_test_pinot_gzip(const uint8_t *in, int n, uint8_t *out, int cap) {
  std::vector<uint8_t> ws(phip::codec::kInflateWs);
  return phip::codec::pinot_gzip_chunk(in, n, out, cap, ws.data());
}

extern "C" int phip_test_inflate_zlib(const uint8_t *in, int n, uint8_t *out, int cap) {
  std::vector<uint8_t> ws(phip::codec::kInflateWs);
  return phip::codec::inflate_zlib(in, n, out, cap, ws.data());
}

extern "C" int phip_test_zstd(const uint8_t *in, int n, uint8_t *out, int cap) {
  std::vector<uint8_t> ws(phip::codec::kZstdWs);
  std::vector<uint8_t> lits(cap > 0 ? cap : 1);
  return phip::codec::zstd_decompress(in, n, out, cap, lits.data(), cap, ws.data());
}
