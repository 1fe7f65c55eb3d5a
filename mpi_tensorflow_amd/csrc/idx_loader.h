#pragma once
#include <stdint.h>

#include <string>
#include <vector>

struct IdxHeader {
  uint32_t magic = 0;
  std::vector<uint32_t> dims;
};

IdxHeader idx_header(const std::string& path);
std::vector<uint8_t> idx_read_u8(const std::string& path, long long start, long long stop,
                                 IdxHeader* hdr_out);
std::vector<float> idx_read_images_f32(const std::string& path, long long start, long long stop,
                                       float pixel_depth);
