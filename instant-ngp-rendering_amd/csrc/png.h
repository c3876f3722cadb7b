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
// First channel as 16-bit values (stbi_load_16(..., 1) as the reference's depth loader calls it,
// src/nerf_loader.cu:629: 16-bit samples as stored, 8-bit ones scaled by 257).
bool decode_png16_file(const std::string& path, std::vector<uint16_t>& gray, int& width, int& height, std::string& err);
// 8-bit PNG of comp (1-4) interleaved channels, rows top to bottom (stbi_write_png as write_stbi calls it,
// src/common_host.cu:240; filter 0, zlib level 6 -- the pixels round-trip, the file bytes are not stb's).
bool encode_png_memory(const uint8_t* pixels, int width, int height, int comp, std::vector<uint8_t>& out, std::string& err);
bool encode_png_file(const std::string& path, const uint8_t* pixels, int width, int height, int comp, std::string& err);

}  // namespace ngp
