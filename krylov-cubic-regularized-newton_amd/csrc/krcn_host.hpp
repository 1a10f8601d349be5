// krcn_host.hpp — what the host-only parts of libkrcn.so share (the C ABI and
// the error recorder), without the HIP headers: the svmlight parser and the
// virtual-rank rendezvous also build with g++ and the host sanitizers
// (Makefile targets asan / tsan, tests/test_sanitizers.py).
#pragma once
#include "krcn.h"

// Records the message of the failing call (krcn_last_error_string) and returns s.
krcn_status fail(krcn_status s, const char* fmt, ...);
