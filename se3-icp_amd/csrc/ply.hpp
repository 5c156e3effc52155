// ply.hpp — minimal PLY point reader for the CLI (open3d::io::CreatePointCloudFromFile
// as used at examples/run_registration_method.cpp:27-31: vertex x/y/z only).
#pragma once
#include <string>
#include <vector>

namespace se3icp {

// Reads vertex x,y,z (any numeric PLY type) into xyz (AoS f64).  Supports ascii,
// binary_little_endian and binary_big_endian.  Returns false with `err` set on failure.
bool read_ply_xyz(const std::string& path, std::vector<double>& xyz, std::string& err);

}  // namespace se3icp
