// raftgpu_internal.h — device-side layout shared by the kernels and the host runtime.
// Layout rationale: DESIGN.md §2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rg {

constexpr uint32_t MAX_R = 8;
constexpr uint64_t BANK_BIT = 1ull << 63;
constexpr uint64_t TERM_MASK = BANK_BIT - 1;

enum : uint32_t {
  M_LOCAL_TICK = 0, M_ELECTION = 1, M_LEADER_HEARTBEAT = 2, M_NOOP = 4, M_PROPOSE = 7,
  M_CHECK_QUORUM = 10, M_REPLICATE = 12, M_REPLICATE_RESP = 13, M_REQUEST_VOTE = 14,
  M_REQUEST_VOTE_RESP = 15, M_INSTALL_SNAPSHOT = 16, M_HEARTBEAT = 17, M_HEARTBEAT_RESP = 18
};
enum : uint32_t { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum : uint32_t { RETRY = 0, WAIT = 1, REPLICATE = 2, SNAPSHOT = 3 };
enum : uint32_t { ENTRY_APP = 0, ENTRY_CONFIG = 1 };
enum : uint32_t { ERR_CONFLICT = 1, ERR_BEYOND = 2, ERR_RING = 4, ERR_CRC = 8, ERR_EMPTY_SNAP = 16 };

// One replica's scalar + remote state: 384 B, double-buffered across ticks.
struct __attribute__((aligned(16))) RepState {
  uint64_t term, vote, leader, committed, applied, last, marker, marker_term;  // 0..63
  uint64_t snap_index, snap_term, cap_base, _r0;                               // 64..95
  uint32_t role, etick, htick, rand_to, rng_ctr, granted, responded, active;   // 96..127
  uint32_t err, drops, _r1[6];                                                 // 128..159
  uint64_t match[MAX_R];                                                       // 160..223
  uint64_t next[MAX_R];                                                        // 224..287
  uint64_t rsnap[MAX_R];                                                       // 288..351
  uint8_t rstate[MAX_R];                                                       // 352..359
  uint8_t _pad[24];                                                            // 360..383
};
static_assert(sizeof(RepState) == 384, "RepState layout");

// 64-byte message slot = rg_msg_view.
struct __attribute__((aligned(16))) MsgHdr {
  uint64_t w0;  // type | from<<8 | to<<16 | reject<<24 | nent<<32
  uint64_t term, log_term, log_index, commit, hint, hint_high;
  uint64_t w7;  // src_a | src_b<<32
};
static_assert(sizeof(MsgHdr) == 64, "MsgHdr layout");

struct TickParams {
  uint32_t G, R, nrep, L, P, E, K, nslab;
  uint32_t ET, HT, CQ, SE, CO, drop_ppm;
  uint32_t flags, crc_const;
  uint64_t seed, tick;
  const RepState* st_in;
  RepState* st_out;
  uint64_t* term_ring;  // [nrep][L]
  uint2* info;          // [2][nrep][L] {crc, type<<24 | len}
  uint8_t* pay;         // [2][nrep][L][P]
  const MsgHdr* hdr_in;
  MsgHdr* hdr_out;          // [nrep][R][K]
  const uint64_t* mt_in;
  uint64_t* mt_out;         // [nrep][R][K][E]
  const uint32_t* cnt_in;
  uint32_t* cnt_out;        // [nrep][R]
  const uint8_t* slabs;     // [nslab][G][E][P]
  const uint8_t* prop_target;
  const uint32_t* prop_count;
  const uint8_t* campaign;
  const uint8_t* isolate;
  const uint32_t* crc_tab;  // [16][256] slice tables + [6][4][256] shift tables
};

// CRC-32/IEEE tables: T[k][b] = raw CRC of byte b followed by k zero bytes (k = 0..15);
// S[j][q][b] = the raw state (b << 8q) advanced through 16·2^j zero bytes (j = 0..5).
constexpr uint32_t CRC_T_WORDS = 16 * 256;
constexpr uint32_t CRC_S_WORDS = 6 * 4 * 256;

// host-side launchers (raftgpu_kernels.hip)
hipError_t launch_tick(const TickParams& p, hipStream_t s, int grid);
hipError_t launch_bootstrap(const TickParams& p, hipStream_t s);
hipError_t launch_fill_slabs(uint8_t* slabs, uint32_t nslab, uint32_t G, uint32_t E, uint32_t P, uint64_t seed,
                             hipStream_t s);
hipError_t launch_sum_committed(const RepState* st, uint32_t G, uint32_t R, unsigned long long* out,
                                hipStream_t s);
hipError_t launch_traffic(const TickParams& p, const RepState* st_prev, unsigned long long* out6, hipStream_t s);
int tick_lds_bytes(uint32_t P);
int tick_blocks_per_cu(uint32_t P);

}  // namespace rg
