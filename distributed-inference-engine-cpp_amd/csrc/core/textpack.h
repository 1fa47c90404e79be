// 4-bit packing of JSON number-list text for the host -> device copy.
//
// A ResNet request carries ~1.05 MB of "0.1234,0.5678,..." text.  With device decode the bytes go
// over PCIe as-is, and that copy (≈22 µs per request at ~47 GB/s) sits on the critical path of
// every batch: it has to finish before the batch's forward can start.  Number lists use at most
// 16 distinct bytes, so the worker packs two characters per byte while it scans the body (the scan
// replaced a plain memcpy into pinned staging), halving the copy; a device kernel expands the
// nibbles back into text right before the decode kernels (kernels/decode.hip).
//
// Alphabet (nibble -> byte): 0-9 -> '0'-'9', 10 ',', 11 '.', 12 '-', 13 '+', 14 'e', 15 ' '.
// Any other byte (e.g. 'E', '\n', '\t') makes pack_nibbles() fail and the caller sends raw text.
// The low nibbles of the six non-digit bytes (C, E, D, B, 5, 0) are distinct, which is what lets
// the AVX2 path classify a byte with one table lookup plus an equality check.
#pragma once

#include <cstddef>
#include <cstdint>

namespace die {

// Packs n bytes of text into (n + 1) / 2 bytes at dst (char 2k in the low nibble of byte k, an odd
// tail padded with ' ').  Returns false, with dst contents unspecified, if a byte is outside the
// alphabet.
bool pack_nibbles(const char* src, size_t n, uint8_t* dst);

// Inverse of pack_nibbles: n characters from (n + 1) / 2 packed bytes.
void unpack_nibbles(const uint8_t* src, size_t n, char* dst);

}  // namespace die
