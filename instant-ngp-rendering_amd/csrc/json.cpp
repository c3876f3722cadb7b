// json.cpp — recursive-descent JSON parser (comments allowed, as json::parse(f, nullptr, true, true)).
#include "json.h"

#include <cmath>
#include <cstdio>
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

}  // namespace ngp
