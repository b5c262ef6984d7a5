// raftgpu_wire.h — parameter block and launchers of the inter-rank message exchange
// (raftgpu_wire.hip; format and protocol in DESIGN.md §6).
#pragma once
#include "raftgpu_internal.h"

namespace rg {

struct WireParams {
  uint32_t G, R, nrep, L, P, E, K;
  Placement pl;
  // sender side: the last tick's outbox (the next tick's *_in) and the sender rings
  const uint64_t* hdr;
  const uint64_t* mt;
  const uint32_t* cnt;
  const uint2* info;       // [2 banks][nrep][L] {slot crc, stream position}
  const uint8_t* pool;      // payload pages, through pt[nrep][PTS]
  const uint32_t* pt;
  uint32_t PTS, maxc;       // stream pages per replica, longest Cmd
  const uint8_t* slabs;     // proposal slabs [nslab][nrep][E][P]: a forwarded Propose ships its Cmds
  const uint2* slab_info;   // [nslab][nrep][E] {SYN_OFF or arena chunk, len}
  const uint8_t* cmds;      // caller Cmd arenas [nslab][cmd_cap]
  uint64_t cmd_cap;
  uint32_t nslab;
  const uint32_t* umap;  // [U] send units s<<28 | d<<24 | j, grouped by destination rank
  const uint32_t* ubeg;  // [N+1] first send unit of each destination
  uint32_t U;
  uint32_t* usize;       // [U] 16-B units of each send unit
  uint64_t* uoff;        // [U+1] exclusive scan of usize
  uint64_t* bsum;        // scan scratch
  uint8_t* send;         // caller's send buffer
  uint64_t send_region[MAX_RANKS];  // byte offset of each destination's region
  uint64_t send_cap[MAX_RANKS];     // fixed-capacity exchange: region bytes (0: sized by the plan); units past it are dropped
  uint64_t* sneed;                  // [N] region bytes the plan asked for, per destination (pack_kernel)
  uint64_t* rneed;                  // [N] the same, per source, from the received region headers (unpack_kernel)
  unsigned long long* drops;        // messages dropped because their unit did not fit its region (cumulative)
  // receiver side
  const uint32_t* rmap;  // [RU] receive units, grouped by source rank (each source's send order)
  const uint32_t* rbeg;  // [N+1]
  uint32_t RU;
  const uint8_t* recv;   // caller's receive buffer
  uint64_t recv_region[MAX_RANKS];
  uint64_t recv_total;   // bytes of the receive buffer in use (end of the last region)
  uint64_t* rhdr;        // remote inbox, TickParams layout
  uint64_t* rmt;
  uint32_t* rcnt;
};

inline uint64_t wire_table_bytes(uint64_t units) { return (units * 8 + 255) & ~255ull; }
// a region: [256-B header: u64 bytes the sender's plan asked for][unit table][data]
constexpr uint64_t WIRE_HDR = 256;
inline uint64_t wire_region_min(uint64_t units) { return units ? WIRE_HDR + wire_table_bytes(units) : 0; }

// plan: usize, the scan, and bounds[r] = uoff[ubeg[r]] (r = 0..N, device) for the region sizes
hipError_t launch_wire_plan(const WireParams& w, uint64_t* bounds, hipStream_t s);
hipError_t launch_wire_pack(const WireParams& w, hipStream_t s);
hipError_t launch_wire_unpack(const WireParams& w, hipStream_t s);

}  // namespace rg
