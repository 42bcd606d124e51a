// sha256.h — SHA-256 (FIPS 180-4) of a byte buffer, for the net identity
// check: Stockfish names its nets nn-<first 12 hex digits of the file's
// SHA-256>.nnue and its `make net` deletes a downloaded file whose digest does
// not match the name ([ref] build.rs:7 EVAL_FILE = nn-ad9b42354671.nnue,
// build.rs:100-112 "Deleted corrupted network file").
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

namespace fnnue {

void sha256(const uint8_t* data, size_t len, uint8_t out[32]);
std::string hex_lower(const uint8_t* bytes, size_t n);

// If the basename of `path` is nn-<12 lowercase hex>.nnue, that prefix;
// otherwise an empty string (the file makes no identity claim).
std::string net_name_digest_prefix(const std::string& path);

}  // namespace fnnue
