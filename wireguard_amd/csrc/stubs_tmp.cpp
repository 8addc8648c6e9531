// TEMPORARY: replaced by gro_host.cpp
#include "../../include/wgcsum.h"
#include "wgcs_ctx.h"
extern "C" {
int wgcs_handle_gro(wgcs_ctx* ctx, uint8_t**, size_t*, size_t*, int, int, int, int*, int*) { return wgcs::set_err(ctx, WGCS_ERR_INVALID_ARG, "not implemented"); }
}
