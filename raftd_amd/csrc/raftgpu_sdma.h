// raftgpu_sdma.h — the copy-back's device-to-host leg on an SDMA engine (raftgpu_sdma.cpp).
#pragma once
#include <cstdint>
#include <string>

namespace rg {

struct SdmaCopier;
// the GPU agent at HIP device `device`'s PCI location and the CPU agent; two completion slots
int sdma_open(int device, SdmaCopier** out, std::string* why);
// asynchronous copy of `bytes` from device memory to pinned host memory on slot 0 or 1
int sdma_copy(SdmaCopier* c, int slot, void* dst_host, const void* src_dev, uint64_t bytes);
// block until the slot's last copy has completed (no-op if none)
void sdma_wait(SdmaCopier* c, int slot);
void sdma_close(SdmaCopier* c);

}  // namespace rg
