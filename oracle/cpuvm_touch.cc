// Reference-accounting build of the CPU baseline (see cpuvm.cc, GKCPU_TOUCH):
// the engine runtime compiled a second time in its own namespace with the
// devrt.h GK_TOUCH_* hooks recording referenced nodes and strings.
// TEST / MEASUREMENT INFRASTRUCTURE, never the product path.
#define GKCPU_TOUCH 1
#define gk gk_touch
#define gk_args gk_args_touch
#include "cpuvm.cc"
