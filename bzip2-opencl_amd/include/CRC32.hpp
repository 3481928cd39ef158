// bz2mi -- bzip2's CRC-32 (MSB-first, polynomial 0x04c11db7), same interface
// as the reference's CRC32 class (include/CRC32.hpp:30-92).  The lookup table
// is computed at compile time instead of being listed.
#ifndef CRC32_HPP
#define CRC32_HPP

#include <array>
#include <cstddef>
#include <cstdint>

namespace bz2mi_detail
{
constexpr std::array<uint32_t, 256> crcTable()
{
    std::array<uint32_t, 256> t{};
    for (uint32_t b = 0; b < 256; ++b)
    {
        uint32_t r = b << 24;
        for (int bit = 0; bit < 8; ++bit)
            r = (r & 0x80000000u) ? (r << 1) ^ 0x04c11db7u : (r << 1);
        t[b] = r;
    }
    return t;
}
inline constexpr std::array<uint32_t, 256> kCrcTable = crcTable();
} // namespace bz2mi_detail

class CRC32
{
    uint32_t reg_ = 0xffffffffu;

public:
    // complemented register, as the stream stores it
    int getCRC() const { return static_cast<int>(~reg_); }

    void updateCRC(int value)
    {
        reg_ = (reg_ << 8) ^ bz2mi_detail::kCrcTable[((reg_ >> 24) ^ static_cast<uint32_t>(value)) & 0xffu];
    }

    // `count` copies of `value` (a run)
    void updateCRC(int value, int count)
    {
        for (; count > 0; --count)
            updateCRC(value);
    }

    void update(const uint8_t *p, size_t n)
    {
        for (size_t i = 0; i < n; ++i)
            updateCRC(p[i]);
    }

    void reset() { reg_ = 0xffffffffu; }
};

#endif
