// gs_changes.cpp -- per-window change emission (placeholder, see below).
#include "gs_internal.hpp"

namespace gsi {
int change_tracking_reset(gs_summary* h, bool full) {
  (void)h;
  (void)full;
  return GS_OK;
}
}  // namespace gsi
