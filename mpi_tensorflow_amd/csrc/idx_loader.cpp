// Native IDX (MNIST) reader: the data-loader half of the tutorial helpers the
// reference imports (`extract_data`, `extract_labels`,
// /root/reference/mpipy.py:12, :215-218).  zlib's gzread handles both the
// gzipped distribution files and raw IDX files.  Reads only the rows a rank
// owns ([start, stop)), decompressing the stream once, and converts pixels to
// float32 (x - 127.5) / 255 in the same pass.
#include "idx_loader.h"

#include <zlib.h>

#include <cstring>
#include <stdexcept>

namespace {

struct GzFile {
  gzFile f;
  explicit GzFile(const std::string& path) : f(gzopen(path.c_str(), "rb")) {
    if (!f) throw std::runtime_error("cannot open " + path);
    gzbuffer(f, 1 << 20);
  }
  ~GzFile() { gzclose(f); }
  void read(void* dst, size_t n, const std::string& path) {
    char* p = static_cast<char*>(dst);
    while (n > 0) {
      unsigned chunk = (unsigned)(n > (1u << 30) ? (1u << 30) : n);
      int got = gzread(f, p, chunk);
      if (got <= 0) throw std::runtime_error(path + ": truncated IDX file");
      p += got;
      n -= (size_t)got;
    }
  }
  void skip(size_t n, const std::string& path) {
    char buf[1 << 16];
    while (n > 0) {
      size_t c = n > sizeof(buf) ? sizeof(buf) : n;
      read(buf, c, path);
      n -= c;
    }
  }
};

uint32_t be32(const unsigned char* b) {
  return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}

}  // namespace

IdxHeader idx_header(const std::string& path) {
  GzFile g(path);
  unsigned char b[4];
  g.read(b, 4, path);
  IdxHeader h;
  h.magic = be32(b);
  if ((h.magic >> 8) != 0x08) throw std::runtime_error(path + ": not a ubyte IDX file");
  int nd = h.magic & 0xFF;
  for (int i = 0; i < nd; ++i) {
    g.read(b, 4, path);
    h.dims.push_back(be32(b));
  }
  return h;
}

std::vector<uint8_t> idx_read_u8(const std::string& path, long long start, long long stop,
                                 IdxHeader* hdr_out) {
  IdxHeader h = idx_header(path);
  if (start < 0 || stop < start || (uint64_t)stop > h.dims.at(0))
    throw std::runtime_error(path + ": row range out of bounds");
  size_t rec = 1;
  for (size_t i = 1; i < h.dims.size(); ++i) rec *= h.dims[i];
  GzFile g(path);
  g.skip(4 + 4 * h.dims.size() + (size_t)start * rec, path);
  std::vector<uint8_t> out((size_t)(stop - start) * rec);
  if (!out.empty()) g.read(out.data(), out.size(), path);
  if (hdr_out) *hdr_out = h;
  return out;
}

std::vector<float> idx_read_images_f32(const std::string& path, long long start, long long stop,
                                       float pixel_depth) {
  std::vector<uint8_t> raw = idx_read_u8(path, start, stop, nullptr);
  std::vector<float> out(raw.size());
  const float half = pixel_depth / 2.0f;
  for (size_t i = 0; i < raw.size(); ++i) out[i] = ((float)raw[i] - half) / pixel_depth;
  return out;
}
