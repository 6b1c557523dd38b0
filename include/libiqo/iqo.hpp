#pragma once

// Umbrella header, as libiqo's include/libiqo/iqo.hpp.
#include <libiqo/LinearResizer.hpp>
#include <libiqo/AreaResizer.hpp>
#include <libiqo/LanczosResizer.hpp>
