// The opaque StackDeviceMemory handle of the C ABI (include/dietgpu_c.h),
// shared by the product library (capi.cpp) and the test-hook library
// (testhooks.hip).
#pragma once

#include "dietgpu/StackDeviceMemory.h"
#include "dietgpu_c.h"

struct dietgpu_stack {
  dietgpu::StackDeviceMemory* mem;
};
