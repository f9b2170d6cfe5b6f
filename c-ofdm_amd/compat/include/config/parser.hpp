// config/parser.hpp — drop-in for the reference's config/parser.hpp:8-10
// (ConfigMap + parse_config). Same rules as config/parser.cpp:4-33: trim,
// skip blank / '#' lines and lines without '=', drop all spaces in key and
// value, std::stol the value; "Cannot open config file" runtime_error.
#pragma once
#include <algorithm>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>

using ConfigMap = std::unordered_map<std::string, long>;

ConfigMap parse_config(const std::string& filename);
