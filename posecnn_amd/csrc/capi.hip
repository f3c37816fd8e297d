// C-ABI housekeeping entry points of libposecnn_hip.so (see include/posecnn_hip.h).
#include "pcnn_common.h"

extern "C" int pcnn_abi_version(void) { return 2; }

extern "C" const char* pcnn_strerror(int code) {
  switch (code) {
    case PCNN_OK: return "ok";
    case PCNN_EINVAL: return "invalid argument";
    case PCNN_EHIP: return "HIP runtime error";
    case PCNN_ECAPACITY: return "workspace or output capacity too small";
    default: return "unknown error";
  }
}
