// ply.cpp — see ply.hpp.
#include "ply.hpp"

#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>

namespace se3icp {

namespace {

struct Prop {
    std::string name;
    std::string type;       // scalar type, or list item type
    std::string count_type; // non-empty for list properties
};
struct Elem {
    std::string name;
    long long count = 0;
    std::vector<Prop> props;
};

int type_size(const std::string& t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "int32" || t == "uint32" || t == "float" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    return 0;
}

double decode(const unsigned char* p, const std::string& t, bool swap) {
    unsigned char b[8];
    const int n = type_size(t);
    for (int i = 0; i < n; ++i) b[i] = swap ? p[n - 1 - i] : p[i];
    if (t == "char" || t == "int8") { int8_t v; std::memcpy(&v, b, 1); return v; }
    if (t == "uchar" || t == "uint8") { uint8_t v; std::memcpy(&v, b, 1); return v; }
    if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return v; }
    if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return v; }
    if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return v; }
    if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return v; }
    if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
    double v;
    std::memcpy(&v, b, 8);
    return v;
}

}  // namespace

bool read_ply_xyz(const std::string& path, std::vector<double>& xyz, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "cannot open " + path; return false; }
    std::string line;
    std::getline(f, line);
    if (line.rfind("ply", 0) != 0) { err = "not a PLY file: " + path; return false; }
    std::string format;
    std::vector<Elem> elems;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string tok;
        ss >> tok;
        if (tok == "format") ss >> format;
        else if (tok == "element") { Elem e; ss >> e.name >> e.count; elems.push_back(e); }
        else if (tok == "property") {
            if (elems.empty()) { err = "property before element"; return false; }
            Prop p;
            std::string t;
            ss >> t;
            if (t == "list") ss >> p.count_type >> p.type >> p.name;
            else { p.type = t; ss >> p.name; }
            elems.back().props.push_back(p);
        } else if (tok == "end_header") break;
    }
    const bool ascii = format == "ascii";
    const bool be = format == "binary_big_endian";
    if (!ascii && !be && format != "binary_little_endian") { err = "unsupported PLY format " + format; return false; }
    for (const Elem& e : elems) {
        if (e.name != "vertex") {
            // skip a preceding element
            for (long long i = 0; i < e.count; ++i) {
                if (ascii) { std::getline(f, line); continue; }
                for (const Prop& p : e.props) {
                    if (!p.count_type.empty()) {
                        unsigned char cb[8];
                        f.read((char*)cb, type_size(p.count_type));
                        const long long cnt = (long long)decode(cb, p.count_type, be);
                        f.seekg(cnt * type_size(p.type), std::ios::cur);
                    } else {
                        f.seekg(type_size(p.type), std::ios::cur);
                    }
                }
            }
            continue;
        }
        int ix = -1, iy = -1, iz = -1;
        for (size_t k = 0; k < e.props.size(); ++k) {
            if (!e.props[k].count_type.empty()) { err = "list property on vertex"; return false; }
            if (e.props[k].name == "x") ix = (int)k;
            if (e.props[k].name == "y") iy = (int)k;
            if (e.props[k].name == "z") iz = (int)k;
        }
        if (ix < 0 || iy < 0 || iz < 0) { err = "vertex element lacks x/y/z"; return false; }
        xyz.resize(3 * (size_t)e.count);
        std::vector<double> row(e.props.size());
        std::vector<unsigned char> buf;
        size_t rec = 0;
        for (const Prop& p : e.props) rec += type_size(p.type);
        buf.resize(rec);
        for (long long i = 0; i < e.count; ++i) {
            if (ascii) {
                if (!std::getline(f, line)) { err = "truncated PLY"; return false; }
                std::istringstream ss(line);
                for (size_t k = 0; k < row.size(); ++k) ss >> row[k];
            } else {
                if (!f.read((char*)buf.data(), rec)) { err = "truncated PLY"; return false; }
                size_t o = 0;
                for (size_t k = 0; k < row.size(); ++k) {
                    row[k] = decode(buf.data() + o, e.props[k].type, be);
                    o += type_size(e.props[k].type);
                }
            }
            xyz[3 * i] = row[ix];
            xyz[3 * i + 1] = row[iy];
            xyz[3 * i + 2] = row[iz];
        }
        return true;
    }
    err = "PLY file has no vertex element";
    return false;
}

}  // namespace se3icp
