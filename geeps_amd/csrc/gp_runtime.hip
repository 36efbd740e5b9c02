// gp_runtime.hip — the C-ABI's runtime helpers (include/gp_reduce.h: devices,
// memory, streams, events) and its inter-process device memory (IPC), so that
// libgeeps' host C++ never names a HIP type.  No kernels here: the kernels and
// their launch logic are gp_reduce.hip; the thread's gp_last_error message is
// set through gp_internal::set_error (defined there).
//
// The IPC handles below wrap the runtime's.  What the runtime's handle names
// on this image (ROCm 7.2, HSA_ENABLE_IPC_MODE_LEGACY=0, DMA-buf IPC), read
// off exported handles by scripts/probes/ipc_handle_layout.py
// (profiles/r06/ipc/handle_layout.json):
//   bytes  0..7   the exporter's device address of the buffer
//   bytes  8..11  the exporter's process id
//   bytes 32..39  the allocation's size
//   bytes 48..51  the exporter's process id again (HIP's part of the handle)
// Nothing in it identifies the allocation beyond (pid, address): ROCr resolves
// a handle when the peer OPENS it, by asking the exporter process -- its own
// server thread on the abstract unix socket "hsa<pid>" -- for a DMA-buf of
// whatever it holds at that address then (libhsa-runtime64.so.1.18.70200:
// the "xhsa%i" / "%li" strings, connect + recvmsg on the attach side, accept +
// strtoull + a map lookup + sendmsg(SCM_RIGHTS) in the server thread).  So a
// handle is only as good as the exporter's address map at open time; libgeeps
// never frees an exported buffer while it runs (oplogs are retired, master
// versions kept), never unmaps a mapping before Shutdown (an address that had
// held a closed mapping was what the runtime misresolved: DESIGN.md §4), and
// checks every mapping against a tag before any of its bytes is used.

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "gp_reduce.h"

namespace gp_internal {
int set_error(int code, const char *msg);
}

namespace {

int set_error(int code, const std::string &msg) { return gp_internal::set_error(code, msg.c_str()); }

#define GP_HIP_TRY(expr)                                                    \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess) {                                                 \
      /* the runtime keeps a failed call's error as the thread's last   */ \
      /* error: clear it, or the next launch's hipGetLastError() check  */ \
      /* reports it (a refused IPC export failed a later sum, round 5)  */ \
      (void)hipGetLastError();                                              \
      return set_error(GP_ERR_HIP, std::string(#expr) + ": " +             \
                                       hipGetErrorString(e_));             \
    }                                                                       \
  } while (0)

constexpr int kMaxDevices = 64;

// Large buffers (libgeeps' oplogs, master versions, staging buckets, caches)
// are asked for physically contiguous first: over 8 fresh 36-GiB arenas after
// random spacers the 8-way sweep sum ran 84.5-86.8 % of 8 TB/s (mean 86.0 %)
// contiguous against 83.1-87.1 % (mean 85.3 %) from plain hipMalloc
// (scripts/tune/contig_tune.hip, profiles/r02/tune/contig_tune.txt).  When the
// device has no contiguous range left, plain hipMalloc.
constexpr size_t kContiguousMin = 64u << 20;

// A buffer meant for IPC (gp_ipc_get_handle) is an allocation of its own,
// rounded up to a multiple of 2 MiB, whose last kIpcTagBytes hold a tag that
// the export writes and every mapping checks.  On MI355X (ROCm 7.2,
// scripts/probes/ipc_probe.py) a process's FIRST device allocation could not
// always be exported: in some runs hipIpcGetMemHandle refused it ("invalid
// argument", persistently), in one run the export succeeded and the peer's
// mapping held other memory, not the exported bytes; every later allocation
// exported and mapped correctly in thousands of tries.  The tag turns a
// mapping of the wrong memory into a loud error instead of silently wrong rows
// (DESIGN.md §4).
constexpr size_t kIpcBlock = 2u << 20;
constexpr size_t kIpcTagBytes = 256;  // the tag's slot at the end of the allocation

std::mutex g_ipc_prime_mu;
bool g_ipc_primed[kMaxDevices];   // g_ipc_prime_mu
void *g_ipc_primer[kMaxDevices];  // g_ipc_prime_mu: kept for the process's lifetime

// The handle as it crosses the C-ABI (GP_IPC_HANDLE_BYTES): the runtime's
// handle, where the allocation's tag lies (bytes from its base), the tag, and
// the allocation base as the exporter saw it.  tag[0] = "gpIP" << 32 | the
// exporter's pid, tag[1] = a hash of (process salt, base, size): a mapping's
// tag names the process and the allocation it really maps.
struct IpcHandleOut {
  hipIpcMemHandle_t h;
  uint64_t tag_offset;
  uint64_t tag[2];
  uint64_t base;
};
static_assert(sizeof(IpcHandleOut) == GP_IPC_HANDLE_BYTES, "IPC handle size");
constexpr uint32_t kIpcTagMagic = 0x67704950u;  // "gpIP"

// One process's IPC calls run one at a time (libgeeps exports and maps from
// several threads: server threads export master versions, reader threads map
// a peer's versions and oplogs); they run once per buffer.
std::mutex g_ipc_mu;
hipStream_t g_ipc_stream[kMaxDevices];  // g_ipc_mu: the tag copies' stream per device

// Every mapping this process holds (g_ipc_mu), by address: what it maps, so
// that a mis-mapping can be told apart as a second reference to a live mapping
// (same address back) or a fresh mapping of other memory.
struct LiveMapping {
  uint32_t pid;
  uint64_t base, bytes;
  uint64_t tag[2];
};
std::map<void *, LiveMapping> g_ipc_live;

// Mis-mappings stay mapped (never used): unmapped, their address would go to
// this process's next allocation, and a handle to a buffer at an address that
// had held a closed mapping is what the runtime was seen to resolve to stale
// memory (round 6 audit).  Counted (gp_ipc_mismaps); past
// kIpcMaxMismaps every
// later open is refused (libgeeps then moves the rows by socket): a runtime
// that keeps mis-mapping is not retried forever.
constexpr int kIpcMaxMismaps = 16;
int g_ipc_mismaps = 0;  // g_ipc_mu

int ipc_stream(hipStream_t *s) {
  int dev = 0;
  GP_HIP_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return set_error(GP_ERR_INVALID, "device id out of range");
  if (!g_ipc_stream[dev]) GP_HIP_TRY(hipStreamCreateWithFlags(&g_ipc_stream[dev], hipStreamNonBlocking));
  *s = g_ipc_stream[dev];
  return GP_OK;
}

// The allocation's tag: the same for every export of it, distinct per process,
// allocation and size.
void ipc_tag(const void *base, size_t bytes, uint64_t tag[2]) {
  static const uint64_t salt = [] {
    uint64_t x = (uint64_t)getpid() * 0x9e3779b97f4a7c15ull;
    x ^= (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    return x;
  }();
  uint64_t h = salt ^ (reinterpret_cast<uintptr_t>(base) * 0xbf58476d1ce4e5b9ull) ^ (bytes * 0x94d049bb133111ebull);
  h ^= h >> 31;
  tag[0] = (uint64_t)kIpcTagMagic << 32 | (uint32_t)getpid();
  tag[1] = h;
}

// The runtime handle's fields as this image lays them out (file header).
struct RuntimeFields {
  uint64_t addr;
  uint32_t pid;
  uint64_t size;
};
RuntimeFields runtime_fields(const hipIpcMemHandle_t &h) {
  const unsigned char *b = reinterpret_cast<const unsigned char *>(&h);
  RuntimeFields f{};
  std::memcpy(&f.addr, b, 8);
  std::memcpy(&f.pid, b + 8, 4);
  std::memcpy(&f.size, b + 32, 8);
  return f;
}

std::string hex_bytes(const void *p, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s;
  const unsigned char *b = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; ++i) {
    s += d[b[i] >> 4];
    s += d[b[i] & 15];
  }
  return s;
}

// "exporter pid P base B (S B); runtime handle: pid P' address A size S'"
// plus whether the two agree, i.e. whether the handle names the buffer libgeeps
// exported.
std::string describe(const IpcHandleOut &in) {
  const RuntimeFields f = runtime_fields(in.h);
  const uint32_t pid = (uint32_t)in.tag[0];
  const uint64_t bytes = in.tag_offset + kIpcTagBytes;
  char buf[320];
  std::snprintf(buf, sizeof buf,
                "exporter pid %u base %#llx (%llu B), tag %016llx %016llx; runtime handle: pid %u address %#llx "
                "size %llu (%s)",
                pid, (unsigned long long)in.base, (unsigned long long)bytes, (unsigned long long)in.tag[0],
                (unsigned long long)in.tag[1], f.pid, (unsigned long long)f.addr, (unsigned long long)f.size,
                f.pid == pid && f.addr == in.base && f.size == bytes ? "names the exported buffer"
                                                                    : "DOES NOT name the exported buffer");
  return buf;
}

// What a mis-mapping holds, from the tag it read: another process's tagged
// buffer (whose pid the tag carries), one this process already maps (and
// where), or untagged memory.
std::string describe_read(const uint64_t got[2], void *p) {
  std::string s;
  char buf[200];
  if ((uint32_t)(got[0] >> 32) == kIpcTagMagic) {
    std::snprintf(buf, sizeof buf, "the mapping holds a buffer tagged by pid %u", (uint32_t)got[0]);
    s = buf;
    for (const auto &kv : g_ipc_live)
      if (kv.second.tag[0] == got[0] && kv.second.tag[1] == got[1]) {
        std::snprintf(buf, sizeof buf, ", the buffer this process maps at %p (pid %u base %#llx)", kv.first,
                      kv.second.pid, (unsigned long long)kv.second.base);
        s += buf;
      }
  } else {
    s = "the mapping holds no libgeeps tag there";
  }
  auto it = g_ipc_live.find(p);
  if (it != g_ipc_live.end()) {
    std::snprintf(buf, sizeof buf, "; the runtime returned the address of a LIVE mapping of pid %u base %#llx",
                  it->second.pid, (unsigned long long)it->second.base);
    s += buf;
  } else {
    s += "; a new address (no live mapping of this process there)";
  }
  return s;
}

}  // namespace

extern "C" {

int gp_device_count(int *count) {
  if (!count) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipGetDeviceCount(count));
  return GP_OK;
}

int gp_set_device(int device) {
  GP_HIP_TRY(hipSetDevice(device));
  return GP_OK;
}

int gp_get_device(int *device) {
  if (!device) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipGetDevice(device));
  return GP_OK;
}

int gp_malloc_device(void **ptr, size_t bytes) {
  if (!ptr) return set_error(GP_ERR_INVALID, "null pointer");
  *ptr = nullptr;
  if (bytes == 0) return GP_OK;
  if (bytes >= kContiguousMin &&
      hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocContiguous) == hipSuccess && *ptr)
    return GP_OK;
  (void)hipGetLastError();  // a failed contiguous request is not this call's error
  *ptr = nullptr;
  GP_HIP_TRY(hipMalloc(ptr, bytes));
  return GP_OK;
}

int gp_malloc_device_shared(void **ptr, size_t bytes) {
  if (!ptr) return set_error(GP_ERR_INVALID, "null pointer");
  *ptr = nullptr;
  if (bytes == 0) return GP_OK;
  // Before a device's first shareable buffer: one throwaway export, so no
  // real buffer is the process's first export -- the buffer the probe saw
  // fail.  The throwaway stays allocated for the process's lifetime, as in the
  // probe's "primed" scenario (scripts/probes/ipc_probe.py): freed, its range
  // could go to the next real buffer, and a handle names an address (file
  // header).  A precaution; what guarantees no wrong rows is the tag check,
  // and a refused export or a failed mapping costs a resend over the socket,
  // not the job (libgeeps' NACKs, wire.hpp).
  int dev = 0;
  GP_HIP_TRY(hipGetDevice(&dev));
  if (dev >= 0 && dev < kMaxDevices) {
    std::lock_guard<std::mutex> lk(g_ipc_prime_mu);
    if (!g_ipc_primed[dev]) {
      g_ipc_primed[dev] = true;
      void *d = nullptr;
      if (hipMalloc(&d, kIpcBlock) == hipSuccess) {
        hipIpcMemHandle_t h;
        (void)hipIpcGetMemHandle(&h, d);
        g_ipc_primer[dev] = d;
      }
      (void)hipGetLastError();  // a refused throwaway export is expected, not this call's error
    }
  }
  return gp_malloc_device(ptr, (bytes + kIpcTagBytes + kIpcBlock - 1) / kIpcBlock * kIpcBlock);
}

int gp_free_device(void *ptr) {
  if (ptr) GP_HIP_TRY(hipFree(ptr));
  return GP_OK;
}

int gp_malloc_host(void **ptr, size_t bytes) {
  if (!ptr) return set_error(GP_ERR_INVALID, "null pointer");
  *ptr = nullptr;
  if (bytes == 0) return GP_OK;
  GP_HIP_TRY(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
  return GP_OK;
}

int gp_free_host(void *ptr) {
  if (ptr) GP_HIP_TRY(hipHostFree(ptr));
  return GP_OK;
}

int gp_host_register(void *ptr, size_t bytes) {
  if (!ptr) return set_error(GP_ERR_INVALID, "null pointer");
  if (bytes == 0) return GP_OK;
  GP_HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return GP_OK;
}

int gp_host_unregister(void *ptr) {
  if (ptr) GP_HIP_TRY(hipHostUnregister(ptr));
  return GP_OK;
}

int gp_memcpy_async(void *dst, const void *src, size_t bytes, gp_stream s) {
  if (bytes == 0) return GP_OK;
  if (!dst || !src) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)s));
  return GP_OK;
}

int gp_memset_async(void *dst, int value, size_t bytes, gp_stream s) {
  if (bytes == 0) return GP_OK;
  if (!dst) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipMemsetAsync(dst, value, bytes, (hipStream_t)s));
  return GP_OK;
}

int gp_stream_create(gp_stream *s) {
  if (!s) return set_error(GP_ERR_INVALID, "null pointer");
  hipStream_t st = nullptr;
  GP_HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  *s = (gp_stream)st;
  return GP_OK;
}

int gp_stream_destroy(gp_stream s) {
  if (s) GP_HIP_TRY(hipStreamDestroy((hipStream_t)s));
  return GP_OK;
}

int gp_stream_synchronize(gp_stream s) {
  GP_HIP_TRY(hipStreamSynchronize((hipStream_t)s));
  return GP_OK;
}

int gp_device_synchronize(void) {
  GP_HIP_TRY(hipDeviceSynchronize());
  return GP_OK;
}

int gp_event_create(gp_event *e) {
  if (!e) return set_error(GP_ERR_INVALID, "null pointer");
  hipEvent_t ev = nullptr;
  GP_HIP_TRY(hipEventCreate(&ev));
  *e = (gp_event)ev;
  return GP_OK;
}

int gp_event_destroy(gp_event e) {
  if (e) GP_HIP_TRY(hipEventDestroy((hipEvent_t)e));
  return GP_OK;
}

int gp_event_record(gp_event e, gp_stream s) {
  GP_HIP_TRY(hipEventRecord((hipEvent_t)e, (hipStream_t)s));
  return GP_OK;
}

int gp_event_synchronize(gp_event e) {
  GP_HIP_TRY(hipEventSynchronize((hipEvent_t)e));
  return GP_OK;
}

int gp_event_elapsed_ms(float *ms, gp_event start, gp_event stop) {
  if (!ms) return set_error(GP_ERR_INVALID, "null pointer");
  GP_HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return GP_OK;
}

int gp_stream_wait_event(gp_stream s, gp_event e) {
  if (!e) return set_error(GP_ERR_INVALID, "null event");
  GP_HIP_TRY(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0));
  return GP_OK;
}

int gp_device_pci_bus_id(int device, char *buf, int len) {
  if (!buf || len < 2) return set_error(GP_ERR_INVALID, "null or short buffer");
  GP_HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
  buf[len - 1] = 0;
  return GP_OK;
}

int gp_ipc_get_handle(void *handle_out, void *device_base) {
  if (!handle_out || !device_base) return set_error(GP_ERR_INVALID, "null pointer");
  std::lock_guard<std::mutex> lk(g_ipc_mu);
  // a handle names a whole allocation: an interior pointer would map the
  // allocation's base in the peer, at the wrong rows
  void *base = nullptr;
  size_t bytes = 0;
  GP_HIP_TRY(hipMemGetAddressRange(&base, &bytes, device_base));
  if (base != device_base || bytes < kIpcBlock || bytes % kIpcBlock) {
    char msg[200];
    std::snprintf(msg, sizeof msg,
                  "IPC export of %p: %s (allocation %p, %zu B); allocate it with gp_malloc_device_shared",
                  device_base, base != device_base ? "not an allocation base" : "not a gp_malloc_device_shared buffer",
                  base, bytes);
    return set_error(GP_ERR_INVALID, msg);
  }
  IpcHandleOut out{};
  out.tag_offset = bytes - kIpcTagBytes;
  out.base = reinterpret_cast<uintptr_t>(base);
  ipc_tag(base, bytes, out.tag);
  hipStream_t s = nullptr;
  if (const int rc = ipc_stream(&s); rc != GP_OK) return rc;
  GP_HIP_TRY(hipMemcpyAsync(static_cast<char *>(base) + out.tag_offset, out.tag, sizeof out.tag,
                            hipMemcpyHostToDevice, s));
  GP_HIP_TRY(hipStreamSynchronize(s));
  GP_HIP_TRY(hipIpcGetMemHandle(&out.h, device_base));
  std::memcpy(handle_out, &out, sizeof out);
  return GP_OK;
}

int gp_ipc_open_handle(void **device_ptr, const void *handle) {
  if (!device_ptr || !handle) return set_error(GP_ERR_INVALID, "null pointer");
  IpcHandleOut in;
  std::memcpy(&in, handle, sizeof in);
  if ((uint32_t)(in.tag[0] >> 32) != kIpcTagMagic) return set_error(GP_ERR_INVALID, "not a gp_ipc_get_handle handle");
  std::lock_guard<std::mutex> lk(g_ipc_mu);
  if (g_ipc_mismaps >= kIpcMaxMismaps) {
    char msg[160];
    std::snprintf(msg, sizeof msg,
                  "IPC mapping refused: the runtime mis-mapped %d handles in this process (kept mapped, unused); "
                  "the limit is %d",
                  g_ipc_mismaps, kIpcMaxMismaps);
    return set_error(GP_ERR_HIP, msg);
  }
  void *p = nullptr;
  GP_HIP_TRY(hipIpcOpenMemHandle(&p, in.h, hipIpcMemLazyEnablePeerAccess));
  // the mapping must span the tag (else it is not the exported allocation:
  // refused without reading past it) and hold the exporter's tag there
  uint64_t got[2] = {0, 0};
  bool read = false;
  hipStream_t s = nullptr;
  int rc = ipc_stream(&s);
  std::string why;
  void *mbase = nullptr;
  size_t mbytes = 0;
  const bool ranged = hipMemGetAddressRange(&mbase, &mbytes, p) == hipSuccess;
  if (!ranged) (void)hipGetLastError();  // no range for this mapping: the tag check below still runs
  const uintptr_t from_base = reinterpret_cast<uintptr_t>(p) - reinterpret_cast<uintptr_t>(mbase);
  if (rc == GP_OK && ranged && (from_base > mbytes || mbytes - from_base < in.tag_offset + sizeof got)) {
    char msg[200];
    std::snprintf(msg, sizeof msg,
                  "IPC mapping %p spans %zu B from %p, short of the exporter's tag at +%llu: the runtime mapped "
                  "other memory than the exported buffer",
                  p, mbytes, mbase, (unsigned long long)in.tag_offset);
    why = msg;
    rc = GP_ERR_HIP;
  }
  if (rc == GP_OK) {
    if (hipMemcpyAsync(got, static_cast<char *>(p) + in.tag_offset, sizeof got, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      (void)hipGetLastError();
      why = "reading the IPC mapping's tag failed";
      rc = GP_ERR_HIP;
    } else {
      read = true;
    }
  }
  if (rc == GP_OK && (got[0] != in.tag[0] || got[1] != in.tag[1])) {
    char msg[240];
    std::snprintf(msg, sizeof msg,
                  "IPC mapping %p does not hold the exporter's tag at +%llu (read %016llx %016llx, expected "
                  "%016llx %016llx)",
                  p, (unsigned long long)in.tag_offset, (unsigned long long)got[0], (unsigned long long)got[1],
                  (unsigned long long)in.tag[0], (unsigned long long)in.tag[1]);
    why = msg;
    rc = GP_ERR_HIP;
  }
  if (rc != GP_OK) {
    // The diagnosis, in the error: whether the handle libgeeps sent names the
    // exported buffer (its runtime fields against the exporter's own record),
    // what the mapping holds instead, whether the runtime handed back a live
    // mapping's address, and the raw runtime handle.
    why += "; " + describe(in);
    if (read) why += "; " + describe_read(got, p);
    why += "; runtime handle " + hex_bytes(&in.h, sizeof in.h);
    // kept mapped, never used (above); counted and bounded
    ++g_ipc_mismaps;
    why += "; kept mapped, unused";
    (void)hipGetLastError();  // no failed call's error may linger into a later launch check
    return set_error(GP_ERR_HIP, why);
  }
  g_ipc_live[p] = LiveMapping{(uint32_t)in.tag[0], in.base, in.tag_offset + kIpcTagBytes, {in.tag[0], in.tag[1]}};
  *device_ptr = p;
  return GP_OK;
}

int gp_ipc_close_handle(void *device_ptr) {
  std::lock_guard<std::mutex> lk(g_ipc_mu);
  if (!device_ptr) return GP_OK;
  g_ipc_live.erase(device_ptr);
  GP_HIP_TRY(hipIpcCloseMemHandle(device_ptr));
  return GP_OK;
}

int gp_ipc_describe_handle(const void *handle, char *buf, int len) {
  if (!handle || !buf || len < 2) return set_error(GP_ERR_INVALID, "null pointer or short buffer");
  IpcHandleOut in;
  std::memcpy(&in, handle, sizeof in);
  if ((uint32_t)(in.tag[0] >> 32) != kIpcTagMagic) return set_error(GP_ERR_INVALID, "not a gp_ipc_get_handle handle");
  const std::string s = describe(in);
  std::snprintf(buf, (size_t)len, "%s", s.c_str());
  return GP_OK;
}

int gp_ipc_mismaps(int *count) {
  if (!count) return set_error(GP_ERR_INVALID, "null pointer");
  std::lock_guard<std::mutex> lk(g_ipc_mu);
  *count = g_ipc_mismaps;
  return GP_OK;
}

}  // extern "C"
