// PNG output, HW2/main.cpp:43-57 semantics: each channel of Pixel::get_color() is
// clamp(int(c / weight), 0, 255) with weight 1 (HW2/Pixel.h:17-28; int() truncates toward
// zero, NaN -> INT_MIN on x86 -> 0 after the clamp), alpha 255.  The reference encodes with
// lodepng 20180114 (HW2/lodepng/); we write 8-bit RGB through zlib.  The decoded pixels are
// identical; the file bytes (colour type, compression) may differ, as lodepng picks a colour
// type automatically.
#include <zlib.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <ios>
#include <stdexcept>
#include <string>
#include <vector>

namespace rt {
namespace {

void be32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(uint8_t(x >> 24));
  v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}

void chunk(std::vector<uint8_t>& file, const char* type, const std::vector<uint8_t>& data) {
  be32(file, (uint32_t)data.size());
  const size_t start = file.size();
  file.insert(file.end(), type, type + 4);
  file.insert(file.end(), data.begin(), data.end());
  const uLong crc = crc32(0L, file.data() + start, (uInt)(file.size() - start));
  be32(file, (uint32_t)crc);
}

// x86-64 cvttss2si: truncation; NaN and out-of-range give INT_MIN ("integer indefinite").
inline int truncate_like_x86(float c) {
  if (!(c > -2147483648.0f && c < 2147483648.0f)) return INT_MIN;
  return (int)c;
}

}  // namespace

uint8_t quantize_channel(float c) {
  const int v = truncate_like_x86(c);
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

void write_png(const std::string& path, const float* rgb, int w, int h) {
  if (w <= 0 || h <= 0) throw std::invalid_argument("png: bad size");
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (1 + 3 * (size_t)w));
  for (int y = 0; y < h; y++) {
    raw.push_back(0);  // filter: none
    for (int x = 0; x < 3 * w; x++) raw.push_back(quantize_channel(rgb[(size_t)y * 3 * w + x]));
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK)
    throw std::runtime_error("png: zlib failure");
  z.resize(zlen);
  std::vector<uint8_t> file = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  std::vector<uint8_t> ihdr;
  be32(ihdr, (uint32_t)w);
  be32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, truecolour, deflate, no filter, no interlace
  chunk(file, "IHDR", ihdr);
  chunk(file, "IDAT", z);
  chunk(file, "IEND", {});
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::ios_base::failure("png: cannot open " + path);
  const size_t n = std::fwrite(file.data(), 1, file.size(), f);
  std::fclose(f);
  if (n != file.size()) throw std::ios_base::failure("png: short write " + path);
}

}  // namespace rt
