// crc32c.hip — host-side CRC-32C (Castagnoli) for checkpoint I/O (include/rst.h rst_crc32c).
// TF tensor bundles checksum every tensor's bytes and every SSTable block with CRC-32C
// (tensorflow/core/util/tensor_bundle, core/lib/io/table); realtime_style_transfer_amd/tf_checkpoint.py
// reads and writes that format (tracing/checkpoint.py:21-37, save_weights /
// load_weights of predict_using_checkpoint.py:84). Slicing-by-8 table implementation.
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../../include/rst.h"

namespace {
struct Crc32cTables {
    uint32_t t[8][256];
    Crc32cTables() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            t[0][i] = c;
        }
        for (int s = 1; s < 8; ++s)
            for (uint32_t i = 0; i < 256; ++i) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
};
const Crc32cTables& tables() {
    static const Crc32cTables T;
    return T;
}
}  // namespace

unsigned int rst_crc32c_extend(unsigned int crc, const void* data, size_t n) {
    const auto& T = tables().t;
    const unsigned char* p = static_cast<const unsigned char*>(data);
    uint32_t c = ~crc;
    while (n >= 8) {
        uint32_t lo, hi;
        std::memcpy(&lo, p, 4);
        std::memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
            T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xFF];
    return ~c;
}
