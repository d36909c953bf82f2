// capi_common.h -- error plumbing shared by the C-ABI translation units.
#pragma once
#include "../../include/openge_hip.h"

// Records the message as the thread's last error (and the context's, when given) and
// returns `code` so call sites can `return oge_fail(...)`.
int oge_fail(oge_ctx *ctx, int code, const char *msg);
