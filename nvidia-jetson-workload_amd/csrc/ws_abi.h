// Helpers shared by the C-ABI entry points of separate translation units (ws_runtime.cpp,
// ws_bvort.hip): one thread-local last-error slot, one exception-to-status mapping.
#pragma once

#include <functional>
#include <stdexcept>
#include <string>

namespace ws {

// Thrown inside an ABI call; abi_guarded maps it to its status code + ws_last_error().
struct AbiError : std::runtime_error {
    int code;
    AbiError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// Runs f, returns WS_OK or the status of what it threw (defined in ws_runtime.cpp).
int abi_guarded(const std::function<void()>& f);
// hipSetDevice after checking a device exists (WS_ERR_DEVICE otherwise; no CPU path).
void abi_set_device(int device);

}  // namespace ws
