// ABI version query.
#include "common.hpp"
extern "C" int sgcn_abi_version(void) { return SGCN_ABI_VERSION; }
