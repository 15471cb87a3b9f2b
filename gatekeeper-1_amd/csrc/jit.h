// Template JIT: a compiled template's predicate bytecode translated to
// straight-line HIP and compiled for gfx950 with hipRTC.
//
// The bytecode VM (kernels.hip) pays an instruction fetch, a dispatch and
// scratch-memory register traffic for every step; the per-template kernel
// binds every VM register to a local (VGPR), turns constants into immediates
// and jumps into direct branches, and calls the same device runtime
// (devrt.h) for the semantics of each instruction — so the two back ends
// agree by construction and the parity tests run both.
#pragma once
#include <string>

#include "compiler.h"
#include "store.h"

namespace gk {

// HIP source of one template kernel named `name` (extern "C" __global__).
std::string jit_source(const Program& p, const CodeBank& bank, const Store& st, const std::string& name);

// Compiles `src` for gfx950 (hipRTC).  Thread-safe; results are cached per
// process by source text and, when GKGPU_JIT_CACHE names a directory (default
// $HOME/.cache/gkgpu-jit; "0" disables), on disk.  Returns false with `log`
// holding the compiler diagnostics.
bool jit_compile(const std::string& src, std::string& code, std::string& log);

// Kernel name for a source body: "gk_t_<16 hex digits of a content hash>".
std::string jit_name(const Program& p, const CodeBank& bank, const Store& st);


}  // namespace gk
