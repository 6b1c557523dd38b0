// TEST INFRASTRUCTURE ONLY (tests/native/asan.mk): the device side of the C ABI as a machine with no
// gfx950 device sees it, so the drop-in classes (libiqo_amd/csrc/resizers.cpp) can be linked into a
// host-only AddressSanitizer / UBSan build with the product's own host code (plan.cpp,
// cpu_generic.cpp) and no HIP runtime: iqo_hip_available() reports no device, every plan call
// returns IQO_HIP_ENODEV, and the classes take their CPU backend -- the path the reference takes
// when no SIMD implementation is available (src/IQOLanczosResizer.cpp:33).
#include <hip/hip_runtime_api.h>

#include "iqo_hip.h"

extern "C" {

int iqo_hip_available(void) { return 0; }
const char *iqo_hip_strerror(int status) { return status ? "no device (host-only sanitizer build)" : "ok"; }
int iqo_hip_plan_lanczos(unsigned, size_t, size_t, size_t, size_t, size_t, int, iqo_hip_plan **p)
{
    *p = nullptr;
    return IQO_HIP_ENODEV;
}
int iqo_hip_plan_area(size_t, size_t, size_t, size_t, int, iqo_hip_plan **p)
{
    *p = nullptr;
    return IQO_HIP_ENODEV;
}
int iqo_hip_plan_linear(size_t, size_t, size_t, size_t, int, iqo_hip_plan **p)
{
    *p = nullptr;
    return IQO_HIP_ENODEV;
}
void iqo_hip_plan_destroy(iqo_hip_plan *) {}
int iqo_hip_plan_query(const iqo_hip_plan *, iqo_hip_plan_desc *) { return IQO_HIP_ENODEV; }
int iqo_hip_resize(iqo_hip_plan *, size_t, const uint8_t *, size_t, uint8_t *) { return IQO_HIP_ENODEV; }
int iqo_hip_resize_device(iqo_hip_plan *, size_t, size_t, size_t, const uint8_t *, size_t, size_t, uint8_t *, void *)
{
    return IQO_HIP_ENODEV;
}

}  // extern "C"

hipError_t hipGetDevice(int *device)
{
    if (device)
        *device = 0;
    return hipErrorNoDevice;
}
