// image.cpp — util::WriteImage (Util.cpp:39-79): gamma-2 (sqrt), clamp(x*255.999, 0, 255),
// vertical flip, PNG (RGB8) or ASCII PPM. The PNG encoder writes stored (uncompressed) deflate
// blocks; stb_image_write is not copied.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace rt2 {

namespace {

uint32_t Crc32(const uint8_t* p, size_t n, uint32_t crc = 0) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  crc = ~crc;
  for (size_t i = 0; i < n; i++) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

void Be32(std::vector<uint8_t>& o, uint32_t v) {
  o.push_back((uint8_t)(v >> 24));
  o.push_back((uint8_t)(v >> 16));
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}

void Chunk(std::vector<uint8_t>& png, const char* type, const std::vector<uint8_t>& data) {
  Be32(png, (uint32_t)data.size());
  size_t start = png.size();
  png.insert(png.end(), type, type + 4);
  png.insert(png.end(), data.begin(), data.end());
  Be32(png, Crc32(png.data() + start, png.size() - start));
}

// Util.cpp:41-48
inline int ToByte(float c) {
  double g = (double)std::sqrt(c) * 255.999;
  if (!(g >= 0.0)) g = 0.0;  // clamp; NaN -> 0
  if (g > 255.0) g = 255.0;
  return (int)g;
}

}  // namespace

std::vector<uint8_t> EncodePng(const uint8_t* rgb, int w, int h) {
  std::vector<uint8_t> raw;  // filter byte 0 + row
  raw.reserve((size_t)h * ((size_t)w * 3 + 1));
  for (int y = 0; y < h; y++) {
    raw.push_back(0);
    raw.insert(raw.end(), rgb + (size_t)y * w * 3, rgb + (size_t)(y + 1) * w * 3);
  }
  std::vector<uint8_t> z = {0x78, 0x01};
  size_t pos = 0;
  do {
    size_t n = std::min<size_t>(65535, raw.size() - pos);
    bool last = pos + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((uint8_t)(n & 0xFF));
    z.push_back((uint8_t)(n >> 8));
    z.push_back((uint8_t)(~n & 0xFF));
    z.push_back((uint8_t)((~n >> 8) & 0xFF));
    z.insert(z.end(), raw.begin() + (long)pos, raw.begin() + (long)(pos + n));
    pos += n;
  } while (pos < raw.size());
  uint32_t a = 1, b = 0;  // adler32
  for (uint8_t c : raw) {
    a = (a + c) % 65521;
    b = (b + a) % 65521;
  }
  Be32(z, (b << 16) | a);
  std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<uint8_t> ihdr;
  Be32(ihdr, (uint32_t)w);
  Be32(ihdr, (uint32_t)h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
  Chunk(png, "IHDR", ihdr);
  Chunk(png, "IDAT", z);
  Chunk(png, "IEND", {});
  return png;
}

// pixels: float3 per pixel, row 0 = bottom row (RayTracer.cpp:97-102). Output is top-down.
bool WriteImage(const float* pixels, int w, int h, const std::string& path, bool png, std::string& err) {
  std::vector<uint8_t> rgb((size_t)w * h * 3);
  for (int y = 0; y < h; y++) {
    const float* src = pixels + (size_t)y * w * 3;
    uint8_t* dst = rgb.data() + (size_t)(h - 1 - y) * w * 3;  // stbi_flip_vertically_on_write
    for (int i = 0; i < w * 3; i++) dst[i] = (uint8_t)ToByte(src[i]);
  }
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) {
    err = "cannot open " + path + " for writing";
    return false;
  }
  if (png) {
    std::vector<uint8_t> enc = EncodePng(rgb.data(), w, h);
    fwrite(enc.data(), 1, enc.size(), f);
  } else {
    fprintf(f, "P3\n%d %d\n255\n", w, h);
    for (size_t i = 0; i < rgb.size(); i += 3) fprintf(f, "%d %d %d\n", rgb[i], rgb[i + 1], rgb[i + 2]);
  }
  fclose(f);
  return true;
}

}  // namespace rt2
