// Go RE2 (regexp, Go 1.15) subset -> byte DFA for re_match on the GPU.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace gk {

enum RegexStatus { RX_OK = 0, RX_INVALID = 1, RX_UNSUPPORTED = 2 };

// Appends the DFA (layout documented in kernels.hip re_run) to `out` and
// returns RX_OK, or RX_INVALID when Go's regexp.Compile would fail (re_match
// then raises a builtin error), or RX_UNSUPPORTED (CPU fallback).
int compile_regex_dfa(const std::string& pattern, std::vector<uint32_t>& out);

// host-side matcher over the same DFA (tests / diagnostics)
int run_regex_dfa(const uint32_t* dfa, const std::string& text);

// byte-class-compressed copy of a DFA for LDS staging (layout in regex.cc)
bool compress_regex_dfa(const std::vector<uint32_t>& dfa, size_t max_bytes, std::vector<uint8_t>& out, uint32_t& nst,
                        uint32_t& ncls, uint32_t& start, uint32_t& sens);
int run_regex_cdfa(const std::vector<uint8_t>& t, uint32_t nst, uint32_t ncls, uint32_t start, uint32_t sens,
                   const std::string& text);

}  // namespace gk
