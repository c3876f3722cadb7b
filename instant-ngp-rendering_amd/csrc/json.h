// json.h — minimal JSON value for network configs and transforms.json (host only).
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <cstdint>
#include <string>
#include <vector>

namespace ngp {

class Json {
public:
	enum Type { Null, Bool, Number, String, Array, Object, Binary };

	Json() = default;
	Json(bool b) : m_type(Bool), m_bool(b) {}
	Json(double d) : m_type(Number), m_num(d) {}
	Json(int i) : m_type(Number), m_num(i) {}
	Json(unsigned i) : m_type(Number), m_num(i) {}
	Json(const char* s) : m_type(String), m_str(s) {}
	Json(std::string s) : m_type(String), m_str(std::move(s)) {}

	static Json array() { Json j; j.m_type = Array; return j; }
	static Json binary(std::vector<uint8_t> bytes) { Json j; j.m_type = Binary; j.m_bin = std::move(bytes); return j; }
	static Json object() { Json j; j.m_type = Object; return j; }
	static Json parse(const std::string& text);

	Type type() const { return m_type; }
	bool is_null() const { return m_type == Null; }
	bool is_object() const { return m_type == Object; }
	bool is_array() const { return m_type == Array; }
	bool is_number() const { return m_type == Number; }
	bool is_string() const { return m_type == String; }
	bool is_bool() const { return m_type == Bool; }
	bool is_binary() const { return m_type == Binary; }
	const std::vector<uint8_t>& bin() const;

	double num() const;
	bool boolean() const;
	const std::string& str() const;
	size_t size() const { return m_type == Array ? m_arr.size() : (m_type == Object ? m_obj.size() : 0); }

	bool contains(const std::string& k) const { return m_type == Object && m_obj.count(k) > 0; }
	const Json& operator[](const std::string& k) const;
	Json& operator[](const std::string& k);  // creates (object) entries
	const Json& operator[](size_t i) const;
	const Json& operator[](int i) const { return (*this)[(size_t)i]; }
	void push_back(Json v);
	void erase(const std::string& k) { m_obj.erase(k); }
	const std::map<std::string, Json>& items() const { return m_obj; }
	const std::vector<Json>& elements() const { return m_arr; }

	double value(const std::string& k, double def) const { return contains(k) && (*this)[k].is_number() ? (*this)[k].num() : def; }
	bool value(const std::string& k, bool def) const { return contains(k) && (*this)[k].is_bool() ? (*this)[k].boolean() : def; }
	std::string value(const std::string& k, const std::string& def) const {
		return contains(k) && (*this)[k].is_string() ? (*this)[k].str() : def;
	}

	// RFC 7386 merge patch (nlohmann::json::merge_patch), used for "parent" configs.
	void merge_patch(const Json& patch);
	std::string dump() const;  // binary values dump as {"binary_bytes": n}

	// MessagePack (nlohmann::json::to_msgpack / from_msgpack), incl. bin and ext as Binary:
	// the container of the reference's .msgpack / .ingp snapshots (src/testbed.cu:4775-4838).
	std::vector<uint8_t> to_msgpack() const;
	static Json from_msgpack(const uint8_t* data, size_t size);

private:
	Type m_type = Null;
	bool m_bool = false;
	double m_num = 0.0;
	std::string m_str;
	std::vector<uint8_t> m_bin;
	std::vector<Json> m_arr;
	std::map<std::string, Json> m_obj;
};

}  // namespace ngp
