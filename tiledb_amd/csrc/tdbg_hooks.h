// tdbg_hooks.h -- experiment and test hooks (timing ablations, A/B switches,
// fault injection, phase clocks).  They are read from the environment only in
// the experiments build (-DTDBG_EXPERIMENTS: tiledb_amd/libtiledb_amd_exp.so,
// `python tiledb_amd/build.py --experiments`); the product library ignores
// every one of them, so a variable left set in a reader process cannot skip
// a decode stage.
#pragma once
#include <stdlib.h>

#ifdef TDBG_EXPERIMENTS
inline const char* tdbg_hook(const char* name) { return getenv(name); }
#else
inline const char* tdbg_hook(const char*) { return nullptr; }
#endif
inline long tdbg_hook_int(const char* name, long dflt) {
  const char* v = tdbg_hook(name);
  return v ? atol(v) : dflt;
}
