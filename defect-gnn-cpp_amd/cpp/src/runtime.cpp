// runtime.cpp — process-wide libdgn context for the facade.
#include "dgn/runtime.hpp"

#include <cstdlib>
#include <stdexcept>

namespace dgn {

Runtime& runtime() {
    static Runtime rt;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* dev = std::getenv("DGN_DEVICE");
        const int st = dgn_ctx_create(dev ? std::atoi(dev) : 0, &rt.ctx);
        if (st != DGN_OK)
            throw std::runtime_error(std::string("libdgn: cannot create a GPU context: ") + dgn_status_string(st));
    });
    return rt;
}

void check(int status, const char* what) {
    if (status == DGN_OK) return;
    std::string msg = std::string(what) + ": " + dgn_status_string(status);
    if (runtime().ctx) msg += std::string(" (") + dgn_ctx_last_error(runtime().ctx) + ")";
    throw std::runtime_error(msg);
}

}  // namespace dgn
