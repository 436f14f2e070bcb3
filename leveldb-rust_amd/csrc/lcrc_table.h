// Host-side SSTable structure walk used by lcrc_table_scan (see lcrc_table.cpp for the reference map).
#pragma once
#include <stdint.h>

#include <functional>
#include <string>
#include <vector>

namespace lcrc_tbl {

constexpr uint64_t TABLE_MAGIC_NUMBER = 0xdb4775248b80fb57ull;  // format.rs:19
constexpr uint32_t BLOCK_HANDLE_MAX_ENCODED_LENGTH = 20;          // format.rs:11
constexpr uint32_t FOOTER_ENCODED_LENGTH = 2 * BLOCK_HANDLE_MAX_ENCODED_LENGTH + 8;  // format.rs:15
constexpr uint32_t BLOCK_TRAILER_SIZE = 5;                        // format.rs:21

struct Handle {
  uint64_t offset = 0, size = 0;
};

bool get_varint32(const uint8_t*& p, const uint8_t* end, uint32_t& out);
bool get_varint64(const uint8_t*& p, const uint8_t* end, uint64_t& out);
// Each returns nullptr on success or the reference's StatusError::Corruption text.
const char* decode_handle(const uint8_t*& p, const uint8_t* end, Handle& h);
const char* decode_footer(const uint8_t* footer48, Handle& metaindex, Handle& index);
// blk = n + 5 bytes of a stored block; out = its (decompressed) contents
const char* block_contents(const uint8_t* blk, uint64_t n, bool verify, int mode, uint32_t flags,
                           std::vector<uint8_t>& out);
// f(key, value, value_len) per entry in order; returning false stops the walk
const char* block_entries(const std::vector<uint8_t>& data,
                          const std::function<bool(const std::string&, const uint8_t*, uint32_t)>& f);
bool snappy_raw_decompress(const uint8_t* p, size_t n, std::vector<uint8_t>& out);
bool snappy_frame_decode(const uint8_t* p, size_t n, std::vector<uint8_t>& out);

}  // namespace lcrc_tbl
