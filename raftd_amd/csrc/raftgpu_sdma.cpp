// raftgpu_sdma.cpp — the copy-back's PCIe leg on a DMA engine (SDMA) instead of shader code.
//
// r03 measured (profiles/r03b_*, r03d_copywg.txt) that a kernel streaming the gathered committed
// entries into host-mapped memory stalls every kernel beside it: with the copy kernel running,
// control_kernel took 3–4 ms and bulk_kernel 15 ms instead of 0.12 / 1.27 ms, whatever the copy's
// workgroup count (2..32). The runtime's own D2H copies are blit kernels too. An SDMA
// engine moves the bytes without shader instructions: hsa_amd_memory_async_copy from the HSA runtime
// the process already holds (HIP sits on it; PyTorch's copy when torch is loaded), resolved at run
// time like RCCL (raftgpu_rccl.cpp), so the library gains no link-time dependency.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "raftgpu_sdma.h"

namespace rg {
namespace {

struct Hsa {
  hsa_status_t (*iterate_agents)(hsa_status_t (*)(hsa_agent_t, void*), void*);
  hsa_status_t (*agent_get_info)(hsa_agent_t, hsa_agent_info_t, void*);
  hsa_status_t (*signal_create)(hsa_signal_value_t, uint32_t, const hsa_agent_t*, hsa_signal_t*);
  hsa_status_t (*signal_destroy)(hsa_signal_t);
  void (*signal_store_relaxed)(hsa_signal_t, hsa_signal_value_t);
  hsa_signal_value_t (*signal_wait_scacquire)(hsa_signal_t, hsa_signal_condition_t, hsa_signal_value_t, uint64_t,
                                              hsa_wait_state_t);
  hsa_status_t (*async_copy)(void*, hsa_agent_t, const void*, hsa_agent_t, size_t, uint32_t, const hsa_signal_t*,
                             hsa_signal_t);
  bool ok = false;
};

const Hsa* hsa() {
  static Hsa a = [] {
    Hsa x{};
    void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);  // the one HIP already loaded
    if (!h) h = dlopen("libhsa-runtime64.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) return x;
    auto sym = [&](const char* n) { return dlsym(h, n); };
    x.iterate_agents = (decltype(x.iterate_agents))sym("hsa_iterate_agents");
    x.agent_get_info = (decltype(x.agent_get_info))sym("hsa_agent_get_info");
    x.signal_create = (decltype(x.signal_create))sym("hsa_signal_create");
    x.signal_destroy = (decltype(x.signal_destroy))sym("hsa_signal_destroy");
    x.signal_store_relaxed = (decltype(x.signal_store_relaxed))sym("hsa_signal_store_relaxed");
    x.signal_wait_scacquire = (decltype(x.signal_wait_scacquire))sym("hsa_signal_wait_scacquire");
    x.async_copy = (decltype(x.async_copy))sym("hsa_amd_memory_async_copy");
    x.ok = x.iterate_agents && x.agent_get_info && x.signal_create && x.signal_destroy && x.signal_store_relaxed &&
           x.signal_wait_scacquire && x.async_copy;
    return x;
  }();
  return a.ok ? &a : nullptr;
}

struct Find {
  const Hsa* h;
  uint32_t bdf, domain;
  hsa_agent_t gpu{}, cpu{};
  bool have_gpu = false, have_cpu = false;
};

hsa_status_t visit(hsa_agent_t a, void* u) {
  Find* f = static_cast<Find*>(u);
  hsa_device_type_t t;
  if (f->h->agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
    f->cpu = a;
    f->have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) {
    uint32_t bdf = 0, dom = 0;
    f->h->agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    f->h->agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    if (bdf == f->bdf && dom == f->domain) {
      f->gpu = a;
      f->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

struct SdmaCopier {
  const Hsa* h = nullptr;
  hsa_agent_t gpu{}, cpu{};
  hsa_signal_t sig[2]{};
  bool pending[2] = {false, false};
};

int sdma_open(int device, SdmaCopier** out, std::string* why) {
  *out = nullptr;
  const Hsa* h = hsa();
  if (!h) {
    *why = "the HSA runtime's copy entry points are not loadable";
    return -1;
  }
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess) {
    *why = "hipDeviceGetAttribute (PCI location)";
    return -1;
  }
  Find f{h, (uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom};
  h->iterate_agents(visit, &f);
  if (!f.have_gpu || !f.have_cpu) {
    *why = "no HSA agent at the device's PCI location, or no CPU agent";
    return -1;
  }
  SdmaCopier* c = new SdmaCopier();
  c->h = h;
  c->gpu = f.gpu;
  c->cpu = f.cpu;
  for (int i = 0; i < 2; ++i)
    if (h->signal_create(0, 0, nullptr, &c->sig[i]) != HSA_STATUS_SUCCESS) {
      *why = "hsa_signal_create";
      delete c;
      return -1;
    }
  *out = c;
  return 0;
}

int sdma_copy(SdmaCopier* c, int slot, void* dst_host, const void* src_dev, uint64_t bytes) {
  c->h->signal_store_relaxed(c->sig[slot], 1);
  if (c->h->async_copy(dst_host, c->cpu, src_dev, c->gpu, bytes, 0, nullptr, c->sig[slot]) != HSA_STATUS_SUCCESS) {
    c->h->signal_store_relaxed(c->sig[slot], 0);
    return -1;
  }
  c->pending[slot] = true;
  return 0;
}

void sdma_wait(SdmaCopier* c, int slot) {
  if (!c->pending[slot]) return;
  while (c->h->signal_wait_scacquire(c->sig[slot], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
  c->pending[slot] = false;
}

void sdma_close(SdmaCopier* c) {
  if (!c) return;
  for (int i = 0; i < 2; ++i) {
    sdma_wait(c, i);
    c->h->signal_destroy(c->sig[i]);
  }
  delete c;
}

}  // namespace rg
