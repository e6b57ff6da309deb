#pragma once
#include "../opencv.hpp"  // compile-check stub (see ../opencv.hpp)
