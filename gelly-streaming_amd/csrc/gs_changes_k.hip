// gs_changes_k.hip -- change-emission kernels (placeholder).
#include "gs_device.hpp"
