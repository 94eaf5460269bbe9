#include "../../include/tcam_hip.h"
extern "C" int tcam_abi_version(void) { return 2; }
extern "C" const char* tcam_arch(void) { return "gfx950"; }
