// kano_internal.hpp -- what the engine's translation units share beyond the
// C ABI (include/kano_hip.h): accessors of a member context for the
// multi-device group (kano_group.hip).  Defined in kano_hip.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "kano_hip.h"

namespace kano_int {

int ctx_device(const kano_ctx* ctx);
hipStream_t ctx_stream(const kano_ctx* ctx);
int64_t ctx_n(const kano_ctx* ctx);
int64_t ctx_W(const kano_ctx* ctx);
// ctx->err = msg; returns code
int ctx_fail(kano_ctx* ctx, int code, const std::string& msg);
// the context's exchange buffers for nranks ranks: its own [OR | cross |
// NAND] words (3 W u64) and every rank's (3 W nranks u64), device memory
int ctx_exchange_buffers(kano_ctx* ctx, int32_t nranks, void** xw, void** xg);
// an RCCL entry point: from the librccl already mapped into the process
// (torch's), else librccl.so; null without RCCL
void* rccl_symbol(const char* name);

}  // namespace kano_int
