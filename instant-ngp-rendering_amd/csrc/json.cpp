// json.cpp — recursive-descent JSON parser (comments allowed, as json::parse(f, nullptr, true, true)).
#include "json.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <sstream>

namespace ngp {

namespace {
struct Parser {
	const std::string& s;
	size_t i = 0;
	explicit Parser(const std::string& t) : s(t) {}

	[[noreturn]] void fail(const char* what) {
		throw std::runtime_error(std::string("JSON parse error: ") + what + " at offset " + std::to_string(i));
	}
	void ws() {
		while (i < s.size()) {
			const char c = s[i];
			if (c == ' ' || c == '\t' || c == '\n' || c == '\r') ++i;
			else if (c == '/' && i + 1 < s.size() && s[i + 1] == '/') {
				while (i < s.size() && s[i] != '\n') ++i;
			} else if (c == '/' && i + 1 < s.size() && s[i + 1] == '*') {
				i += 2;
				while (i + 1 < s.size() && !(s[i] == '*' && s[i + 1] == '/')) ++i;
				i += 2;
			} else break;
		}
	}
	bool eat(char c) {
		ws();
		if (i < s.size() && s[i] == c) { ++i; return true; }
		return false;
	}
	std::string string_lit() {
		if (!eat('"')) fail("expected string");
		std::string out;
		while (i < s.size() && s[i] != '"') {
			char c = s[i++];
			if (c == '\\') {
				if (i >= s.size()) fail("bad escape");
				const char e = s[i++];
				switch (e) {
					case 'n': out += '\n'; break;
					case 't': out += '\t'; break;
					case 'r': out += '\r'; break;
					case 'b': out += '\b'; break;
					case 'f': out += '\f'; break;
					case 'u': {
						if (i + 4 > s.size()) fail("bad \\u escape");
						const unsigned cp = (unsigned)std::strtoul(s.substr(i, 4).c_str(), nullptr, 16);
						i += 4;
						if (cp < 0x80) out += (char)cp;
						else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
						else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
					} break;
					default: out += e;
				}
			} else out += c;
		}
		if (i >= s.size()) fail("unterminated string");
		++i;
		return out;
	}
	Json value() {
		ws();
		if (i >= s.size()) fail("unexpected end");
		const char c = s[i];
		if (c == '{') {
			++i;
			Json o = Json::object();
			if (eat('}')) return o;
			do {
				ws();
				std::string k = string_lit();
				if (!eat(':')) fail("expected ':'");
				o[k] = value();
			} while (eat(','));
			if (!eat('}')) fail("expected '}'");
			return o;
		}
		if (c == '[') {
			++i;
			Json a = Json::array();
			if (eat(']')) return a;
			do a.push_back(value());
			while (eat(','));
			if (!eat(']')) fail("expected ']'");
			return a;
		}
		if (c == '"') return Json(string_lit());
		if (s.compare(i, 4, "true") == 0) { i += 4; return Json(true); }
		if (s.compare(i, 5, "false") == 0) { i += 5; return Json(false); }
		if (s.compare(i, 4, "null") == 0) { i += 4; return Json(); }
		char* end = nullptr;
		const double d = std::strtod(s.c_str() + i, &end);
		if (end == s.c_str() + i) fail("unexpected character");
		i = (size_t)(end - s.c_str());
		return Json(d);
	}
};
}  // namespace

Json Json::parse(const std::string& text) {
	Parser p(text);
	Json v = p.value();
	p.ws();
	if (p.i != text.size()) p.fail("trailing characters");
	return v;
}

double Json::num() const {
	if (m_type == Bool) return m_bool ? 1.0 : 0.0;
	if (m_type != Number) throw std::runtime_error("JSON value is not a number");
	return m_num;
}
bool Json::boolean() const {
	if (m_type == Number) return m_num != 0.0;
	if (m_type != Bool) throw std::runtime_error("JSON value is not a bool");
	return m_bool;
}
const std::vector<uint8_t>& Json::bin() const {
	if (m_type != Binary) throw std::runtime_error("JSON value is not binary");
	return m_bin;
}
const std::string& Json::str() const {
	if (m_type != String) throw std::runtime_error("JSON value is not a string");
	return m_str;
}
const Json& Json::operator[](const std::string& k) const {
	static const Json null;
	if (m_type != Object) return null;
	auto it = m_obj.find(k);
	return it == m_obj.end() ? null : it->second;
}
Json& Json::operator[](const std::string& k) {
	if (m_type == Null) m_type = Object;
	if (m_type != Object) throw std::runtime_error("JSON value is not an object");
	return m_obj[k];
}
const Json& Json::operator[](size_t i) const {
	if (m_type != Array || i >= m_arr.size()) throw std::runtime_error("JSON array index out of range");
	return m_arr[i];
}
void Json::push_back(Json v) {
	if (m_type == Null) m_type = Array;
	if (m_type != Array) throw std::runtime_error("JSON value is not an array");
	m_arr.push_back(std::move(v));
}
void Json::merge_patch(const Json& patch) {
	if (!patch.is_object()) {
		*this = patch;
		return;
	}
	if (!is_object()) *this = Json::object();
	for (const auto& kv : patch.m_obj) {
		if (kv.second.is_null()) m_obj.erase(kv.first);
		else m_obj[kv.first].merge_patch(kv.second);
	}
}
std::string Json::dump() const {
	std::ostringstream o;
	switch (m_type) {
		case Null: o << "null"; break;
		case Bool: o << (m_bool ? "true" : "false"); break;
		case Number: {
			char buf[64];
			if (std::floor(m_num) == m_num && std::fabs(m_num) < 1e15) std::snprintf(buf, sizeof(buf), "%.0f", m_num);
			else std::snprintf(buf, sizeof(buf), "%.9g", m_num);
			o << buf;
		} break;
		case String: {
			o << '"';
			for (char c : m_str) {
				if (c == '"' || c == '\\') o << '\\' << c;
				else if (c == '\n') o << "\\n";
				else o << c;
			}
			o << '"';
		} break;
		case Array: {
			o << '[';
			for (size_t k = 0; k < m_arr.size(); ++k) o << (k ? "," : "") << m_arr[k].dump();
			o << ']';
		} break;
		case Binary: o << "{\"binary_bytes\":" << m_bin.size() << "}"; break;
		case Object: {
			o << '{';
			bool first = true;
			for (const auto& kv : m_obj) {
				o << (first ? "" : ",") << Json(kv.first).dump() << ':' << kv.second.dump();
				first = false;
			}
			o << '}';
		} break;
	}
	return o.str();
}

// ---------------------------------------------------------------------------
// MessagePack
// ---------------------------------------------------------------------------
namespace {
void put_be(std::vector<uint8_t>& o, uint64_t v, int bytes) {
	for (int k = bytes - 1; k >= 0; --k) o.push_back((uint8_t)(v >> (8 * k)));
}
void put_len(std::vector<uint8_t>& o, size_t n, uint8_t fix_base, size_t fix_max, uint8_t t8, uint8_t t16, uint8_t t32) {
	if (fix_max && n <= fix_max) o.push_back((uint8_t)(fix_base | n));
	else if (t8 && n < 256) { o.push_back(t8); put_be(o, n, 1); }
	else if (n < 65536) { o.push_back(t16); put_be(o, n, 2); }
	else { o.push_back(t32); put_be(o, n, 4); }
}
void encode(const Json& j, std::vector<uint8_t>& o) {
	switch (j.type()) {
		case Json::Null: o.push_back(0xc0); break;
		case Json::Bool: o.push_back(j.boolean() ? 0xc3 : 0xc2); break;
		case Json::Number: {
			const double v = j.num();
			if (std::floor(v) == v && std::fabs(v) < 9.2e18) {
				if (v >= 0) {
					const uint64_t u = (uint64_t)v;
					if (u < 128) o.push_back((uint8_t)u);
					else if (u < 256) { o.push_back(0xcc); put_be(o, u, 1); }
					else if (u < 65536) { o.push_back(0xcd); put_be(o, u, 2); }
					else if (u < 4294967296ull) { o.push_back(0xce); put_be(o, u, 4); }
					else { o.push_back(0xcf); put_be(o, u, 8); }
				} else {
					const int64_t s = (int64_t)v;
					if (s >= -32) o.push_back((uint8_t)(int8_t)s);
					else if (s >= -128) { o.push_back(0xd0); put_be(o, (uint64_t)s, 1); }
					else if (s >= -32768) { o.push_back(0xd1); put_be(o, (uint64_t)s, 2); }
					else if (s >= -2147483648ll) { o.push_back(0xd2); put_be(o, (uint64_t)s, 4); }
					else { o.push_back(0xd3); put_be(o, (uint64_t)s, 8); }
				}
			} else {
				uint64_t bits;
				std::memcpy(&bits, &v, 8);
				o.push_back(0xcb);
				put_be(o, bits, 8);
			}
		} break;
		case Json::String: {
			const std::string& s = j.str();
			put_len(o, s.size(), 0xa0, 31, 0xd9, 0xda, 0xdb);
			o.insert(o.end(), s.begin(), s.end());
		} break;
		case Json::Binary: {
			const auto& b = j.bin();
			put_len(o, b.size(), 0, 0, 0xc4, 0xc5, 0xc6);
			o.insert(o.end(), b.begin(), b.end());
		} break;
		case Json::Array:
			put_len(o, j.size(), 0x90, 15, 0, 0xdc, 0xdd);
			for (const Json& e : j.elements()) encode(e, o);
			break;
		case Json::Object:
			put_len(o, j.size(), 0x80, 15, 0, 0xde, 0xdf);
			for (const auto& kv : j.items()) {
				encode(Json(kv.first), o);
				encode(kv.second, o);
			}
			break;
	}
}
struct Reader {
	const uint8_t* d;
	size_t n, i = 0;
	uint64_t be(int bytes) {
		if (i + bytes > n) throw std::runtime_error("msgpack: truncated");
		uint64_t v = 0;
		for (int k = 0; k < bytes; ++k) v = (v << 8) | d[i++];
		return v;
	}
	std::vector<uint8_t> raw(size_t len) {
		if (i + len > n) throw std::runtime_error("msgpack: truncated");
		std::vector<uint8_t> v(d + i, d + i + len);
		i += len;
		return v;
	}
	std::string str(size_t len) {
		auto v = raw(len);
		return std::string(v.begin(), v.end());
	}
	Json array(size_t len) {
		Json a = Json::array();
		for (size_t k = 0; k < len; ++k) a.push_back(value());
		return a;
	}
	Json map(size_t len) {
		Json m = Json::object();
		for (size_t k = 0; k < len; ++k) {
			Json key = value();
			std::string ks = key.is_string() ? key.str() : key.dump();
			m[ks] = value();
		}
		return m;
	}
	Json value() {
		const uint8_t t = (uint8_t)be(1);
		if (t < 0x80) return Json((double)t);
		if (t >= 0xe0) return Json((double)(int8_t)t);
		if ((t & 0xf0) == 0x80) return map(t & 0x0f);
		if ((t & 0xf0) == 0x90) return array(t & 0x0f);
		if ((t & 0xe0) == 0xa0) return Json(str(t & 0x1f));
		switch (t) {
			case 0xc0: return Json();
			case 0xc2: return Json(false);
			case 0xc3: return Json(true);
			case 0xc4: return Json::binary(raw(be(1)));
			case 0xc5: return Json::binary(raw(be(2)));
			case 0xc6: return Json::binary(raw(be(4)));
			case 0xc7: { const size_t l = be(1); be(1); return Json::binary(raw(l)); }  // ext: subtype dropped
			case 0xc8: { const size_t l = be(2); be(1); return Json::binary(raw(l)); }
			case 0xc9: { const size_t l = be(4); be(1); return Json::binary(raw(l)); }
			case 0xca: { const uint32_t b = (uint32_t)be(4); float f; std::memcpy(&f, &b, 4); return Json((double)f); }
			case 0xcb: { const uint64_t b = be(8); double f; std::memcpy(&f, &b, 8); return Json(f); }
			case 0xcc: return Json((double)be(1));
			case 0xcd: return Json((double)be(2));
			case 0xce: return Json((double)be(4));
			case 0xcf: return Json((double)be(8));
			case 0xd0: return Json((double)(int8_t)be(1));
			case 0xd1: return Json((double)(int16_t)be(2));
			case 0xd2: return Json((double)(int32_t)be(4));
			case 0xd3: return Json((double)(int64_t)be(8));
			case 0xd4: be(1); return Json::binary(raw(1));
			case 0xd5: be(1); return Json::binary(raw(2));
			case 0xd6: be(1); return Json::binary(raw(4));
			case 0xd7: be(1); return Json::binary(raw(8));
			case 0xd8: be(1); return Json::binary(raw(16));
			case 0xd9: return Json(str(be(1)));
			case 0xda: return Json(str(be(2)));
			case 0xdb: return Json(str(be(4)));
			case 0xdc: return array(be(2));
			case 0xdd: return array(be(4));
			case 0xde: return map(be(2));
			case 0xdf: return map(be(4));
			default: throw std::runtime_error("msgpack: unsupported type byte");
		}
	}
};
}  // namespace

std::vector<uint8_t> Json::to_msgpack() const {
	std::vector<uint8_t> o;
	encode(*this, o);
	return o;
}

Json Json::from_msgpack(const uint8_t* data, size_t size) {
	Reader r{data, size};
	Json v = r.value();
	return v;
}

}  // namespace ngp
