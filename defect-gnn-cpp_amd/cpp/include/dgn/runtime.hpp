// runtime.hpp — the facade's process-wide libdgn context (device from $DGN_DEVICE, default 0).
// Calls are serialized with a mutex; a failing status is rethrown as std::runtime_error
// (the reference throws C++ exceptions; nothing is thrown across the extern "C" boundary).
#pragma once
#include <mutex>
#include <string>

#include "dgn.h"

namespace dgn {

struct Runtime {
    dgn_ctx* ctx = nullptr;
    std::mutex mu;
};
Runtime& runtime();
void check(int status, const char* what);  // throws std::runtime_error on status != DGN_OK

}  // namespace dgn
