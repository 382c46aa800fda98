// mj423_internal.h -- helpers shared by the library's host translation units (not exported API).
#pragma once
#include <mutex>
#include <string>

#include "../../include/mj423gpu.h"

// Records msg as this thread's mj423_last_error() and returns code.
int mj423_set_error(int code, const std::string& msg);
// The process-default context behind the reference's context-free symbols
// (idct, ycbcr_to_rgb, mjpeg423_decode); created on first use, nullptr if no GPU.
mj423_ctx* mj423_default_ctx();
// The HIP device a context was created on (-1 for null).
int mj423_ctx_device_id(mj423_ctx* ctx);
// Serialises users of the default context.
std::mutex& mj423_default_mutex();
