// png.cpp — minimal PNG decoder on zlib (the reference decodes with stb_image, src/nerf_loader.cu:520-560).
#include "png.h"

#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>

namespace ngp {

static uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

static int paeth(int a, int b, int c) {
	const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
	if (pa <= pb && pa <= pc) return a;
	return pb <= pc ? b : c;
}

// Unfiltered sample bytes of a non-interlaced PNG (big-endian 16-bit samples kept as bytes).
struct RawPng {
	std::vector<uint8_t> img, plte, trns;
	uint32_t w = 0, h = 0;
	int depth = 0, ctype = 0, channels = 0;
	size_t bpp = 0;
};
static bool decode_png_raw(const uint8_t* d, size_t size, RawPng& out, std::string& err);

bool decode_png_memory(const uint8_t* d, size_t size, std::vector<uint8_t>& rgba, int& width, int& height,
                       std::string& err) {
	RawPng r;
	if (!decode_png_raw(d, size, r, err)) return false;
	const uint32_t w = r.w, h = r.h;
	const int ctype = r.ctype, depth = r.depth;
	const size_t bpp = r.bpp;
	const std::vector<uint8_t>& img = r.img;
	const std::vector<uint8_t>& plte = r.plte;
	const std::vector<uint8_t>& trns = r.trns;
	width = (int)w;
	height = (int)h;
	rgba.assign((size_t)w * h * 4, 255);
	const int step = depth / 8;  // 16-bit: keep the high byte
	for (size_t i = 0; i < (size_t)w * h; ++i) {
		const uint8_t* p = &img[i * bpp];
		uint8_t* o = &rgba[i * 4];
		switch (ctype) {
			case 0: o[0] = o[1] = o[2] = p[0]; break;
			case 2: o[0] = p[0]; o[1] = p[step]; o[2] = p[2 * step]; break;
			case 3: {
				const uint8_t k = p[0];
				if ((size_t)k * 3 + 2 < plte.size()) { o[0] = plte[k * 3]; o[1] = plte[k * 3 + 1]; o[2] = plte[k * 3 + 2]; }
				o[3] = k < trns.size() ? trns[k] : 255;
			} break;
			case 4: o[0] = o[1] = o[2] = p[0]; o[3] = p[step]; break;
			case 6: o[0] = p[0]; o[1] = p[step]; o[2] = p[2 * step]; o[3] = p[3 * step]; break;
		}
	}
	return true;
}

bool decode_png16_file(const std::string& path, std::vector<uint16_t>& gray, int& width, int& height, std::string& err) {
	std::ifstream f(path, std::ios::binary);
	if (!f) { err = "cannot open " + path; return false; }
	std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
	RawPng r;
	if (!decode_png_raw(buf.data(), buf.size(), r, err)) return false;
	if (r.ctype == 3) { err = "palette image as depth"; return false; }
	width = (int)r.w;
	height = (int)r.h;
	gray.resize((size_t)r.w * r.h);
	for (size_t i = 0; i < gray.size(); ++i) {
		const uint8_t* p = &r.img[i * r.bpp];
		gray[i] = r.depth == 16 ? (uint16_t)((p[0] << 8) | p[1]) : (uint16_t)(p[0] * 257u);
	}
	return true;
}

static bool decode_png_raw(const uint8_t* d, size_t size, RawPng& out, std::string& err) {
	static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
	if (size < 8 || std::memcmp(d, sig, 8) != 0) { err = "not a PNG file"; return false; }
	size_t pos = 8;
	uint32_t w = 0, h = 0;
	int depth = 0, ctype = 0, interlace = 0;
	std::vector<uint8_t> idat, plte, trns;
	while (pos + 12 <= size) {
		const uint32_t len = be32(d + pos);
		const char* type = (const char*)d + pos + 4;
		const uint8_t* body = d + pos + 8;
		if (pos + 12 + len > size) { err = "truncated chunk"; return false; }
		if (!std::strncmp(type, "IHDR", 4)) {
			w = be32(body);
			h = be32(body + 4);
			depth = body[8];
			ctype = body[9];
			interlace = body[12];
		} else if (!std::strncmp(type, "IDAT", 4)) idat.insert(idat.end(), body, body + len);
		else if (!std::strncmp(type, "PLTE", 4)) plte.assign(body, body + len);
		else if (!std::strncmp(type, "tRNS", 4)) trns.assign(body, body + len);
		else if (!std::strncmp(type, "IEND", 4)) break;
		pos += 12 + len;
	}
	if (!w || !h) { err = "missing IHDR"; return false; }
	if (interlace) { err = "interlaced PNG unsupported"; return false; }
	if (!(depth == 8 || depth == 16)) { err = "unsupported bit depth"; return false; }
	int channels;
	switch (ctype) {
		case 0: channels = 1; break;
		case 2: channels = 3; break;
		case 3: channels = 1; if (depth != 8) { err = "palette depth"; return false; } break;
		case 4: channels = 2; break;
		case 6: channels = 4; break;
		default: err = "unsupported color type"; return false;
	}
	const size_t bpp = (size_t)channels * (depth / 8);
	const size_t stride = bpp * w;
	std::vector<uint8_t> raw((stride + 1) * h);
	uLongf out_len = (uLongf)raw.size();
	if (uncompress(raw.data(), &out_len, idat.data(), (uLong)idat.size()) != Z_OK || out_len != raw.size()) {
		err = "zlib inflate failed";
		return false;
	}
	std::vector<uint8_t> img(stride * h);
	for (uint32_t y = 0; y < h; ++y) {
		const uint8_t f = raw[y * (stride + 1)];
		const uint8_t* src = &raw[y * (stride + 1) + 1];
		uint8_t* cur = &img[y * stride];
		const uint8_t* prev = y ? &img[(y - 1) * stride] : nullptr;
		for (size_t x = 0; x < stride; ++x) {
			const int a = x >= bpp ? cur[x - bpp] : 0, b = prev ? prev[x] : 0, c = (prev && x >= bpp) ? prev[x - bpp] : 0;
			int v = src[x];
			switch (f) {
				case 0: break;
				case 1: v += a; break;
				case 2: v += b; break;
				case 3: v += (a + b) / 2; break;
				case 4: v += paeth(a, b, c); break;
				default: err = "bad filter"; return false;
			}
			cur[x] = (uint8_t)v;
		}
	}
	out.w = w;
	out.h = h;
	out.depth = depth;
	out.ctype = ctype;
	out.channels = channels;
	out.bpp = bpp;
	out.img.swap(img);
	out.plte.swap(plte);
	out.trns.swap(trns);
	return true;
}

bool decode_png_file(const std::string& path, std::vector<uint8_t>& rgba, int& width, int& height, std::string& err) {
	std::ifstream f(path, std::ios::binary);
	if (!f) { err = "cannot open " + path; return false; }
	std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
	return decode_png_memory(buf.data(), buf.size(), rgba, width, height, err);
}

// PNG encoder (write_stbi's png branch, src/common_host.cu:234-248): 8-bit gray / GA / RGB / RGBA, filter 0 on every
// row, one zlib stream in one IDAT chunk.
static void put_be32(std::vector<uint8_t>& o, uint32_t v) {
	o.push_back((uint8_t)(v >> 24));
	o.push_back((uint8_t)(v >> 16));
	o.push_back((uint8_t)(v >> 8));
	o.push_back((uint8_t)v);
}

static void put_chunk(std::vector<uint8_t>& o, const char* type, const uint8_t* data, size_t n) {
	put_be32(o, (uint32_t)n);
	const size_t start = o.size();
	o.insert(o.end(), type, type + 4);
	if (n) o.insert(o.end(), data, data + n);
	put_be32(o, (uint32_t)crc32(0L, o.data() + start, (uInt)(n + 4)));
}

bool encode_png_memory(const uint8_t* pixels, int width, int height, int comp, std::vector<uint8_t>& out, std::string& err) {
	static const uint8_t ctypes[5] = {0, 0, 4, 2, 6};
	if (width <= 0 || height <= 0 || comp < 1 || comp > 4) {
		err = "encode_png: invalid image shape";
		return false;
	}
	const size_t row = (size_t)width * comp;
	std::vector<uint8_t> raw((row + 1) * (size_t)height);
	for (int y = 0; y < height; ++y) {
		raw[(row + 1) * y] = 0;
		std::memcpy(&raw[(row + 1) * y + 1], pixels + row * y, row);
	}
	uLongf zn = compressBound((uLong)raw.size());
	std::vector<uint8_t> z(zn);
	if (compress2(z.data(), &zn, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
		err = "encode_png: zlib deflate failed";
		return false;
	}
	out.clear();
	static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
	out.insert(out.end(), sig, sig + 8);
	std::vector<uint8_t> ihdr;
	put_be32(ihdr, (uint32_t)width);
	put_be32(ihdr, (uint32_t)height);
	ihdr.push_back(8);
	ihdr.push_back(ctypes[comp]);
	ihdr.push_back(0);
	ihdr.push_back(0);
	ihdr.push_back(0);
	put_chunk(out, "IHDR", ihdr.data(), ihdr.size());
	put_chunk(out, "IDAT", z.data(), zn);
	put_chunk(out, "IEND", nullptr, 0);
	return true;
}

bool encode_png_file(const std::string& path, const uint8_t* pixels, int width, int height, int comp, std::string& err) {
	std::vector<uint8_t> buf;
	if (!encode_png_memory(pixels, width, height, comp, buf, err)) return false;
	std::ofstream f(path, std::ios::binary);
	if (!f) {
		err = "encode_png: cannot open " + path;
		return false;
	}
	f.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)buf.size());
	if (!f) {
		err = "encode_png: write failed for " + path;
		return false;
	}
	return true;
}

}  // namespace ngp
