// ABI version query (SGCN_ABI_DIAG_FLAG set in a diagnostic build: see common.hpp).
#include "common.hpp"
extern "C" int sgcn_abi_version(void) {
  return SGCN_ABI_VERSION | (SGCN_DIAG_BUILD ? SGCN_ABI_DIAG_FLAG : 0);
}
