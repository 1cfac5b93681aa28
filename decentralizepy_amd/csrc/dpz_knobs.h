// Tuning and forced-path switches of the codec kernels.
//
// The product library (libdpzcodec.so) compiles every switch to its measured default: no call
// path reads the environment, so nothing in a node's environment can change which kernels run.
// The diagnostic build (`make diag-lib` or `make all` -> libdpzcodec_diag.so, compiled with -DDPZ_DIAG) reads
// DPZ_<NAME> on every call instead: the A/B measurements under tools/diag and the forced-path GPU
// tests (tests/conftest.py `diag_lib`) load it explicitly.
#pragma once
#include <cstdlib>

#ifdef DPZ_DIAG
#define DPZ_KNOB_STR(name) getenv("DPZ_" #name)
#else
#define DPZ_KNOB_STR(name) ((const char*)nullptr)
#endif
// the integer value of DPZ_<name> (diagnostic build, when set), else dflt
#define DPZ_KNOB_INT(name, dflt) \
  (DPZ_KNOB_STR(name) ? atoll(DPZ_KNOB_STR(name)) : (long long)(dflt))
