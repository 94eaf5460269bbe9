// Placeholder until the permutohedral HIP kernel lands.
#include "common.h"
extern "C" size_t tcam_bilateral_ws_bytes(int N, int H, int W, int K) { return 0; }
extern "C" int tcam_bilateral_batch(const float*, const float*, float*, void*, int, int, int, int,
                                    float, float, int, void*) { return TCAM_E_ARG; }
extern "C" void bilateralfilter_batch(float*, int, float*, int, float*, int, int, int, int, int,
                                      float, float) {}
