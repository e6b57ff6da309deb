// The adapter's one libmim context (device 0, its own HIP stream), shared by the scene path
// (TestsDetector.cpp) and, with MIM_GPU_SIFT, the model loader (ModelsDetector.cpp): the models are
// described once (main.cpp:22) and every scene reuses the same context.
#pragma once
#include "mim.hpp"

inline mim::Detector& mim_device() {
    static mim::Detector det(0);
    return det;
}
