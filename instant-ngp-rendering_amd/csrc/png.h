// png.h — PNG -> RGBA8 decoder (8-bit gray/GA/RGB/RGBA/palette, 16-bit truncated), non-interlaced.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ngp {

// Returns false (with `err`) for unsupported files; the caller may fall back to another decoder.
bool decode_png_file(const std::string& path, std::vector<uint8_t>& rgba, int& width, int& height, std::string& err);
bool decode_png_memory(const uint8_t* data, size_t size, std::vector<uint8_t>& rgba, int& width, int& height,
                       std::string& err);

}  // namespace ngp
