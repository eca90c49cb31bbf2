// Basic types of the host runtime (mirrors aby3/Common/Defines.h).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace aby3 {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i32 = int32_t;
using i64 = int64_t;

// cryptoTools block: 16 bytes, toBlock(hi, lo) = LE64(lo) || LE64(hi).
struct block {
    u64 lo = 0, hi = 0;
    bool operator==(const block& o) const { return lo == o.lo && hi == o.hi; }
    bool operator!=(const block& o) const { return !(*this == o); }
    const u8* data() const { return reinterpret_cast<const u8*>(this); }
    u8* data() { return reinterpret_cast<u8*>(this); }
};
inline block toBlock(u64 hi, u64 lo) { return block{lo, hi}; }
inline block toBlock(u64 lo) { return block{lo, 0}; }
// bytes of a device allocation that is exported through IPC: whole 2 MiB
// blocks (aby3g_ipc_get_handle refuses anything else)
inline size_t ipcBytes(size_t b) {
    const size_t g = (size_t)2 << 20;
    return b ? (b + g - 1) / g * g : g;
}

#define ABY3_STR2(x) #x
#define ABY3_STR(x) ABY3_STR2(x)
#define LOCATION __FILE__ ":" ABY3_STR(__LINE__)
#define RTE_LOC std::runtime_error(LOCATION)

// Decimal places of the fixed-point types (aby3/sh3/Sh3FixedPoint.h:7-13).
enum Decimal { D0 = 0, D8 = 8, D16 = 16, D32 = 32 };

}  // namespace aby3
