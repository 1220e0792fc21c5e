// PNG output, HW2/main.cpp:43-57 semantics: each channel of Pixel::get_color() is
// clamp(int(c / weight), 0, 255) with weight 1 (HW2/Pixel.h:17-28; int() truncates toward
// zero, NaN -> INT_MIN on x86 -> 0 after the clamp), alpha 255, encoded the way the reference's
// lodepng 20180114 (HW2/lodepng/) encodes with its default settings:
//   * colour type and bit depth chosen automatically from the image (auto_convert): a palette
//     when at most 256 colours and it beats grey, in first-appearance order; otherwise grey
//     (bit depth 1/2/4/8, the least that holds every value) or 8-bit RGB;
//   * scanline filters: none for palette or sub-8-bit images, else per row the filter with the
//     least sum of |signed bytes| (lodepng counts a byte s >= 128 as 255 - s), type 0 first;
// so the PNG's header, palette and filtered image data are the reference file's byte for byte
// (tests/test_host.py against PNGs the reference wrote).  Only the deflate stream that carries
// the filtered data differs (zlib here, lodepng's own compressor there): it inflates to the
// same bytes.
#include <zlib.h>

#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <ios>
#include <stdexcept>
#include <string>
#include <unordered_map>
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

// Bits a grey value needs (lodepng's scaling of 1/2/4-bit grey: multiples of 255, 85, 17).
unsigned grey_bits(uint8_t v) {
  if (v == 0 || v == 255) return 1;
  if (v % 17 == 0) return v % 85 == 0 ? 2 : 4;
  return 8;
}

enum : uint8_t { kGrey = 0, kRGB = 2, kPalette = 3 };

struct Mode {
  uint8_t type = kRGB, depth = 8;
  std::vector<uint32_t> palette;  // 0xRRGGBB, first-appearance order
};

// lodepng_get_color_profile + lodepng_auto_choose_color for an opaque RGB8 image.
Mode choose_mode(const std::vector<uint8_t>& rgb, size_t npix,
                 std::unordered_map<uint32_t, uint32_t>& index) {
  bool colored = false;
  unsigned bits = 1;
  std::vector<uint32_t> colors;  // up to 257 distinct colours counted
  for (size_t i = 0; i < npix; i++) {
    const uint8_t r = rgb[3 * i], g = rgb[3 * i + 1], b = rgb[3 * i + 2];
    if (bits < 8) bits = std::max(bits, grey_bits(r));
    if (!colored && (r != g || r != b)) {
      colored = true;
      bits = 8;
    }
    if (colors.size() < 257) {
      const uint32_t c = (uint32_t)r << 16 | (uint32_t)g << 8 | b;
      if (index.emplace(c, (uint32_t)colors.size()).second) colors.push_back(c);
    }
  }
  Mode m;
  const size_t n = colors.size();
  const unsigned pbits = n <= 2 ? 1 : (n <= 4 ? 2 : (n <= 16 ? 4 : 8));
  bool palette = n <= 256 && bits <= 8;
  if (npix < n * 2) palette = false;
  if (!colored && bits <= pbits) palette = false;
  if (palette) {
    m.type = kPalette;
    m.depth = (uint8_t)pbits;
    m.palette = colors;
  } else {
    m.type = colored ? kRGB : kGrey;
    m.depth = (uint8_t)bits;
  }
  return m;
}

uint8_t paeth(int a, int b, int c) {
  const int pa = std::abs(b - c), pb = std::abs(a - c), pc = std::abs(a + b - c - c);
  if (pc < pa && pc < pb) return (uint8_t)c;
  if (pb < pa) return (uint8_t)b;
  return (uint8_t)a;
}

// One scanline through filter `type` (PNG filter method 0; prev == nullptr on the first row).
void filter_line(uint8_t* out, const uint8_t* in, const uint8_t* prev, size_t len, size_t bw,
                 int type) {
  for (size_t i = 0; i < len; i++) {
    const int a = i >= bw ? in[i - bw] : 0, b = prev ? prev[i] : 0,
              c = (prev && i >= bw) ? prev[i - bw] : 0;
    int p = 0;
    if (type == 1) p = a;
    if (type == 2) p = b;
    if (type == 3) p = (a + b) >> 1;
    if (type == 4) p = paeth(a, b, c);
    out[i] = (uint8_t)(in[i] - p);
  }
}

}  // namespace

uint8_t quantize_channel(float c) {
  const int v = truncate_like_x86(c);
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

void write_png(const std::string& path, const float* rgb, int w, int h) {
  if (w <= 0 || h <= 0) throw std::invalid_argument("png: bad size");
  const size_t npix = (size_t)w * h;
  std::vector<uint8_t> q(3 * npix);
  for (size_t i = 0; i < 3 * npix; i++) q[i] = quantize_channel(rgb[i]);
  std::unordered_map<uint32_t, uint32_t> index;
  const Mode m = choose_mode(q, npix, index);
  // unfiltered scanlines in the chosen mode (sub-byte pixels packed MSB first, rows padded)
  const size_t bpp = m.type == kRGB ? 24 : m.depth;
  const size_t line = ((size_t)w * bpp + 7) / 8, bw = (bpp + 7) / 8;
  std::vector<uint8_t> rows(line * (size_t)h, 0);
  for (int y = 0; y < h; y++) {
    uint8_t* row = &rows[(size_t)y * line];
    for (int x = 0; x < w; x++) {
      const uint8_t* p = &q[3 * ((size_t)y * w + x)];
      if (m.type == kRGB) {
        row[3 * x] = p[0], row[3 * x + 1] = p[1], row[3 * x + 2] = p[2];
        continue;
      }
      unsigned v = m.type == kGrey
                       ? (unsigned)(p[0] >> (8 - m.depth))
                       : index.at((uint32_t)p[0] << 16 | (uint32_t)p[1] << 8 | p[2]);
      const size_t bit = (size_t)x * m.depth;
      row[bit / 8] |= (uint8_t)(v << (8 - m.depth - bit % 8));
    }
  }
  // filters: none for palette / sub-8-bit images, else least sum of |signed bytes| per row
  const bool adaptive = m.type != kPalette && m.depth >= 8;
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (1 + line));
  std::vector<uint8_t> tryf[5];
  for (auto& t : tryf) t.resize(line);
  for (int y = 0; y < h; y++) {
    const uint8_t* in = &rows[(size_t)y * line];
    const uint8_t* prev = y ? &rows[(size_t)(y - 1) * line] : nullptr;
    int best = 0;
    if (adaptive) {
      size_t smallest = 0;
      for (int t = 0; t < 5; t++) {
        filter_line(tryf[t].data(), in, prev, line, bw, t);
        size_t sum = 0;
        for (size_t i = 0; i < line; i++) {
          const uint8_t s = tryf[t][i];
          sum += t == 0 ? s : (s < 128 ? s : 255u - s);
        }
        if (t == 0 || sum < smallest) {
          best = t;
          smallest = sum;
        }
      }
    } else {
      filter_line(tryf[0].data(), in, prev, line, bw, 0);
    }
    raw.push_back((uint8_t)best);
    raw.insert(raw.end(), tryf[best].begin(), tryf[best].end());
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
  ihdr.insert(ihdr.end(), {m.depth, m.type, 0, 0, 0});  // deflate, filter method 0, no interlace
  chunk(file, "IHDR", ihdr);
  if (m.type == kPalette) {
    std::vector<uint8_t> plte;
    for (uint32_t c : m.palette) plte.insert(plte.end(), {uint8_t(c >> 16), uint8_t(c >> 8), uint8_t(c)});
    chunk(file, "PLTE", plte);
  }
  chunk(file, "IDAT", z);
  chunk(file, "IEND", {});
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::ios_base::failure("png: cannot open " + path);
  const size_t n = std::fwrite(file.data(), 1, file.size(), f);
  std::fclose(f);
  if (n != file.size()) throw std::ios_base::failure("png: short write " + path);
}

}  // namespace rt
