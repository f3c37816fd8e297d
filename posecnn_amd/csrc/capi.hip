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

namespace pcnn {
thread_local hipEvent_t t_done_event = nullptr;
}

// The next op called on this thread records `event` (a created hipEvent_t)
// when its last kernel completes; see pcnn_common.h launch_last.
extern "C" int pcnn_set_completion_event(void* event) {
  pcnn::t_done_event = (hipEvent_t)event;
  return PCNN_OK;
}

// 1 if the event set by pcnn_set_completion_event was not taken by an op's
// last launch (the op has no completion hook on this path); clears it.
extern "C" int pcnn_completion_event_pending(void) {
  const int p = pcnn::t_done_event != nullptr;
  pcnn::t_done_event = nullptr;
  return p;
}
