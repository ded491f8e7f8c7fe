// Exchange-area layout of the wide persistent launch (kernels_persist_wide.hip), one formula per
// side, shared by the kernel and by the host-side exhaustive check (wide_layout_check, exported
// as wrnn_debug_wide_layout): every producer packet of a hop lands on exactly one consumer
// packet, with the (row, unit) contents the consumer's MFMA B operand expects, inside the
// slot's main region, 16-byte aligned; out-of-range offsets of non-publishing / non-polling
// lanes stay out of range for every buffer and slot. (the round-3 18-row
// instance deadlocked on a packet that was neither a publication nor the reset; this is the
// check that the shipped instance's packets cannot be misplaced.)
#pragma once

namespace wrnn {
namespace wide {

constexpr int kSlots = 32;          // workgroups (slots) per XCD group
constexpr int kWaves = 8;           // waves per workgroup (K-eighths of 64 units)
constexpr int kRows = 16;           // MFMA N columns = rows per group
constexpr int kPackets = 4;         // 16-byte packets per consumer lane and hop (k-steps 4p..4p+3)
// One published vector (x1, h1, x2, h2, y1, y2) per step: two slots (step parity), each
// [e 8][p 4][lane 64] packets of 4 floats in MFMA B-operand order, then 1024 spare floats
constexpr int WS_MAIN = kWaves * kPackets * 64 * 4;
constexpr int WSLOT = WS_MAIN + 1024;
constexpr int WV = 2 * WSLOT;
constexpr int kBufs = 6;            // x1, h1, x2, h2, y1, y2
constexpr int WX_D = kBufs * WV;    // candidates [n 16][slot 32] (value, tag|class)
constexpr int WX_CAND = kRows * kSlots * 2;
constexpr int WX_GROUP = WX_D + WX_CAND + 64;
constexpr unsigned kNoOffset = 0x80000000u;  // lanes without a packet: outside every buffer
constexpr unsigned kRsrcRecords = 0x7fffffffu;  // persist_common.h mk_rsrc num_records

// consumer: byte offset (in a slot) of packet 0 of lane l of wave v; packet i at + 1 KiB i.
// It holds row n = l % 16, units 64 v + 16 (l / 16) + 4 i + q, q < 4.
__host__ __device__ constexpr unsigned cons_off(int v, int l) { return (unsigned)((v * 4 * 64 + l) * 16); }
__host__ __device__ constexpr int cons_row(int l) { return l & 15; }
__host__ __device__ constexpr int cons_unit0(int v, int l, int i) { return 64 * v + 16 * (l >> 4) + 4 * i; }
// producer: byte offset of the packet of the unit quad cul .. cul + 3 (cul % 4 == 0) of row cn,
// published by slot w (units 16 w + cul + q)
__host__ __device__ constexpr unsigned prod_off(int w, int cn, int cul) {
    return (unsigned)((((w >> 2) * 4 + (cul >> 2)) * 64 + 16 * (w & 3) + cn) * 16);
}
// byte offset of buffer hb, parity slot s inside the group's area
__host__ __device__ constexpr unsigned slot_base(int hb, unsigned s) {
    return (unsigned)(hb * WV) * 4u + (s & 1u) * (unsigned)WSLOT * 4u;
}
// candidate of row n from slot w (8 bytes: value, step tag | class)
__host__ __device__ constexpr unsigned cand_off(int n, int w) { return (unsigned)((n * kSlots + w) * 2) * 4u; }

static_assert(WX_GROUP % 4 == 0 && WX_D % 4 == 0, "reset works in 16-byte units");
static_assert(kNoOffset > kRsrcRecords, "the no-packet offset must fail the range check");

}  // namespace wide
}  // namespace wrnn
