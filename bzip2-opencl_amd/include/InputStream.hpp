// bz2mi -- bzip2 decompressing input stream with the reference's interface
// (Stan1slav337/Bzip2-OpenCL include/InputStream.hpp:36-159) and its error
// messages (InputStream.hpp:84,114,121; BlockDecompressor.hpp:111,161,215,248,
// 276; HuffmanStageDecoder.hpp:55; BitInputStream.hpp:47).
//
// Decoding runs on the device (bz2mi_dstream, include/bz2mi.h; SURVEY 8(f)
// row 1) in bounded windows: the input is read in kChunk pieces into a window
// of at least kWindow bytes, every whole block in it is decoded at once
// (Huffman tables, MTF/RLE2, inverse BWT, RLE1 and the block / stream CRCs),
// bytes are served from an output buffer of kOutCap bytes, and the window
// slides on -- host memory stays O(window + output buffer) whatever the input
// size, as the reference's block-at-a-time reader (InputStream.hpp:51-72).
// Errors carry the reference's messages and surface after the bytes of the
// blocks before the failing one.  As in the reference, blocks are
// limited to digit x 10,000 bytes (Config.hpp:30, BlockDecompressor.hpp:
// 158-162) and decoding ends at the first end-of-stream marker
// (InputStream.hpp:136-143).  BZ2MI_BZIP2_COMPAT=1 reads like bzip2 instead:
// digit x 100,000-byte blocks (stock files, bz2mi's 900 KB mode) and every
// concatenated stream.
// BZ2MI_HOST_DECODER=1 selects the host decoder below instead (a block at a
// time, the reference's structure: Huffman tables -> MTF/RLE2 symbols ->
// inverse BWT -> RLE1 expansion with the block CRC checked).
#ifndef INPUT_STREAM_HPP
#define INPUT_STREAM_HPP

#include <algorithm>
#include <cstdint>
#include <istream>
#include <stdexcept>
#include <vector>

#include <cstdlib>
#include <iterator>
#include <string>

#include "CRC32.hpp"
#include "Config.hpp"
#include "bz2mi.h"

class InputStream
{
public:
    explicit InputStream(std::istream &in) : in_(in) {}

    // next byte, or -1 at the end of the stream
    ~InputStream()
    {
        if (dctx_)
            bz2mi_ddestroy(dctx_);
    }
    InputStream(const InputStream &) = delete;
    InputStream &operator=(const InputStream &) = delete;

    int read()
    {
        if (pos_ == len_ && !refill())
            return -1;
        return cur_[pos_++];
    }

    // up to `length` bytes into buffer[offset..]; -1 at the end of the stream
    int read(std::vector<uint8_t> &buffer, int offset, int length)
    {
        int got = 0;
        while (got < length)
        {
            if (pos_ == len_ && !refill())
                break;
            size_t take = len_ - pos_;
            if (take > static_cast<size_t>(length - got))
                take = static_cast<size_t>(length - got);
            for (size_t i = 0; i < take; ++i)
                buffer[offset + got + i] = cur_[pos_ + i];
            pos_ += take;
            got += static_cast<int>(take);
        }
        return got == 0 && length > 0 ? -1 : got;
    }

    void close()
    {
        done_ = true;
        block_.clear();
        out_.clear();
        win_.clear();
        cur_ = nullptr;
        pos_ = len_ = 0;
        if (dctx_)
            bz2mi_ddestroy(dctx_);
        dctx_ = nullptr;
    }

private:
    // ---- bit reader (MSB first)
    uint32_t bits(int n)
    {
        while (have_ < n)
        {
            const int c = in_.get();
            if (c == std::char_traits<char>::eof())
                throw std::runtime_error("Insufficient data");
            acc_ = (acc_ << 8) | static_cast<uint32_t>(c & 0xff);
            have_ += 8;
        }
        have_ -= n;
        return static_cast<uint32_t>((acc_ >> have_) & ((n == 32) ? 0xffffffffull : ((1ull << n) - 1)));
    }
    bool bit() { return bits(1) != 0; }

    void header()
    {
        const uint32_t magic = bits(16), h = bits(8);
        const int digit = static_cast<int>(bits(8)) - '0';
        if (magic != static_cast<uint32_t>(STREAM_START_MARKER_1) || h != static_cast<uint32_t>(STREAM_START_MARKER_2) ||
            digit < 1 || digit > 9)
            throw std::runtime_error("Invalid BZip2 header");
        maxBlock_ = digit * (bzip2Compat() ? BLOCKSIZE_BZIP2 : BLOCKSIZE_DEFAULT);
        started_ = true;
    }

    bool refill()
    {
        if (done_)
            return false;
        if (!modeChosen_)
        {
            modeChosen_ = true;
            const char *h = std::getenv("BZ2MI_HOST_DECODER");
            host_ = h && *h && *h != '0';
        }
        if (!host_)
            return refillDevice();
        const bool got = refillHost();
        cur_ = block_.data();
        len_ = block_.size();
        pos_ = 0;
        return got;
    }

    static bool bzip2Compat()
    {
        const char *e = std::getenv("BZ2MI_BZIP2_COMPAT");
        return e && *e && *e != '0';
    }

    static constexpr size_t kChunk = 16u << 20;    // input read per step
    static constexpr size_t kWindow = 64u << 20;   // window handed to the device (at least)
    static constexpr size_t kOutCap = 64u << 20;   // output buffer (grows if one block needs more)

    // the next window's blocks decoded on the device
    bool refillDevice()
    {
        if (!dctx_)
        {
            int device = 0;
            if (const char *d = std::getenv("BZ2MI_DEVICE"))
                device = std::atoi(d);
            const bool compat = bzip2Compat();
            dctx_ = bz2mi_dcreate(compat ? BLOCKSIZE_BZIP2 : BLOCKSIZE_DEFAULT, device);
            if (!dctx_)
                throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
            if (compat)
                bz2mi_dset_flags(dctx_, BZ2MI_DEC_CONCATENATED);
            window_ = kWindow;
            chunk_ = kChunk;
            size_t outCap = kOutCap;
            if (const char *w = std::getenv("BZ2MI_DSTREAM_WINDOW"))  // tests: many small windows
            {
                window_ = std::max<size_t>(static_cast<size_t>(std::atoll(w)), 64);
                chunk_ = window_ / 4 + 1;
                outCap = window_;
            }
            out_.resize(outCap);
        }
        size_t want = window_;
        for (;;)
        {
            while (!eof_ && win_.size() < want)
            {
                const size_t old = win_.size();
                win_.resize(old + chunk_);
                in_.read(reinterpret_cast<char *>(win_.data() + old), static_cast<std::streamsize>(chunk_));
                win_.resize(old + static_cast<size_t>(in_.gcount()));
                if (!in_)
                    eof_ = true;
            }
            uint64_t end = 0;
            size_t n = 0;
            int fin = 0;
            const int rc = bz2mi_dstream(dctx_, win_.data(), win_.size(), bit_, eof_ ? 1 : 0, out_.data(),
                                         out_.size(), &end, &n, &fin);
            if (rc == BZ2MI_ESPACE)
            {
                out_.resize(n + (n >> 3) + 4096);
                continue;
            }
            if (rc != BZ2MI_OK)
            {
                done_ = true;
                throw std::runtime_error(bz2mi_last_error());
            }
            // slide the window: keep the bytes from the byte holding `end` on
            const size_t byte = static_cast<size_t>(end / 8);
            win_.erase(win_.begin(), win_.begin() + static_cast<std::ptrdiff_t>(byte));
            bit_ = static_cast<unsigned>(end & 7);
            if (fin)
                done_ = true;
            if (n)
            {
                cur_ = out_.data();
                len_ = n;
                pos_ = 0;
                return true;
            }
            if (fin)
                return false;
            if (eof_)  // (a final call decodes something or fails)
            {
                done_ = true;
                throw std::runtime_error("Insufficient data");
            }
            want = win_.size() + window_;  // no whole block in the window yet: a longer one
        }
    }

    bool refillHost()
    {
        if (done_)
            return false;
        if (!started_)
            header();
        block_.clear();
        pos_ = 0;
        const uint32_t m1 = bits(24), m2 = bits(24);
        if (m1 == static_cast<uint32_t>(BLOCK_HEADER_MARKER_1) && m2 == static_cast<uint32_t>(BLOCK_HEADER_MARKER_2))
        {
            const uint32_t crc = decodeBlock();
            streamCRC_ = ((streamCRC_ << 1) | (streamCRC_ >> 31)) ^ crc;
            return !block_.empty() || refillHost();
        }
        if (m1 == static_cast<uint32_t>(STREAM_END_MARKER_1) && m2 == static_cast<uint32_t>(STREAM_END_MARKER_2))
        {
            done_ = true;
            if (bits(32) != streamCRC_)
                throw std::runtime_error("BZip2 stream CRC error");
            return false;
        }
        done_ = true;
        throw std::runtime_error("BZip2 stream format error");
    }

    // one block; fills block_ and returns its stored CRC
    uint32_t decodeBlock()
    {
        const uint32_t storedCRC = bits(32);
        if (bit())
            throw std::runtime_error("BZip2 randomised blocks not implemented");
        const uint32_t origPtr = bits(24);
        // symbol map
        uint8_t symbols[256];
        int k = 0;
        const uint32_t ranges = bits(16);
        for (int r = 0; r < 16; ++r)
            if (ranges & (0x8000u >> r))
            {
                const uint32_t m = bits(16);
                for (int j = 0; j < 16; ++j)
                    if (m & (0x8000u >> j))
                        symbols[k++] = static_cast<uint8_t>(r * 16 + j);
            }
        const int alpha = k + 2;
        const int nTables = static_cast<int>(bits(3));
        const int nSel = static_cast<int>(bits(15));
        if (k == 0 || nTables < HUFFMAN_MINIMUM_TABLES || nTables > HUFFMAN_MAXIMUM_TABLES || nSel < 1)
            throw std::runtime_error("block Huffman tables invalid");
        std::vector<uint8_t> sel(static_cast<size_t>(nSel));
        {
            uint8_t order[HUFFMAN_MAXIMUM_TABLES] = {0, 1, 2, 3, 4, 5};
            for (int s = 0; s < nSel; ++s)
            {
                int j = 0;
                while (bit())
                    if (++j >= nTables)
                        throw std::runtime_error("block Huffman tables invalid");
                const uint8_t v = order[j];
                for (; j > 0; --j)
                    order[j] = order[j - 1];
                order[0] = v;
                sel[static_cast<size_t>(s)] = v;
            }
        }
        // code lengths (delta coded) -> canonical decoding tables
        int len[HUFFMAN_MAXIMUM_TABLES][HUFFMAN_MAXIMUM_ALPHABET_SIZE];
        for (int t = 0; t < nTables; ++t)
        {
            int cur = static_cast<int>(bits(5));
            for (int s = 0; s < alpha; ++s)
            {
                for (;;)
                {
                    if (cur < 1 || cur > HUFFMAN_DECODE_MAXIMUM_CODE_LENGTH)
                        throw std::runtime_error("block Huffman tables invalid");
                    if (!bit())
                        break;
                    cur += bit() ? -1 : 1;
                }
                len[t][s] = cur;
            }
        }
        struct Table
        {
            int minLen, maxLen;
            int32_t limit[HUFFMAN_DECODE_MAXIMUM_CODE_LENGTH + 2];
            int32_t base[HUFFMAN_DECODE_MAXIMUM_CODE_LENGTH + 2];
            uint16_t perm[HUFFMAN_MAXIMUM_ALPHABET_SIZE];
        } tab[HUFFMAN_MAXIMUM_TABLES];
        for (int t = 0; t < nTables; ++t)
        {
            Table &T = tab[t];
            T.minLen = 32;
            T.maxLen = 0;
            for (int s = 0; s < alpha; ++s)
            {
                T.minLen = len[t][s] < T.minLen ? len[t][s] : T.minLen;
                T.maxLen = len[t][s] > T.maxLen ? len[t][s] : T.maxLen;
            }
            int p = 0, code = 0;
            for (int L = T.minLen; L <= T.maxLen; ++L)
            {
                T.base[L] = p - code;  // symbol index = code + base[L]
                for (int s = 0; s < alpha; ++s)
                    if (len[t][s] == L)
                    {
                        T.perm[p++] = static_cast<uint16_t>(s);
                        code++;
                    }
                T.limit[L] = code - 1;  // largest code of this length
                code <<= 1;
            }
        }
        // Huffman -> MTF/RLE2 -> BWT bytes
        std::vector<uint8_t> bwt;
        bwt.reserve(static_cast<size_t>(maxBlock_));
        uint8_t mtf[256];
        for (int i = 0; i < k; ++i)
            mtf[i] = symbols[i];
        uint32_t counts[256] = {0};
        int group = 0, left = 0;
        const Table *T = nullptr;
        uint64_t run = 0;
        int runBit = 0;
        for (;;)
        {
            if (left == 0)
            {
                if (group >= nSel)
                    throw std::runtime_error("Error decoding  block");
                T = &tab[sel[static_cast<size_t>(group++)]];
                left = HUFFMAN_GROUP_RUN_LENGTH;
            }
            left--;
            int L = T->minLen;
            int32_t code = static_cast<int32_t>(bits(L));
            while (code > T->limit[L])
            {
                if (++L > T->maxLen)
                    throw std::runtime_error("Error decoding  block");
                code = (code << 1) | static_cast<int32_t>(bit());
            }
            const int sym = T->perm[code + T->base[L]];
            if (sym <= HUFFMAN_SYMBOL_RUNB)
            {
                run += static_cast<uint64_t>(sym + 1) << runBit;  // bijective base 2
                if (++runBit > 40)
                    throw std::runtime_error("BZip2 block exceeds declared block size");
                continue;
            }
            if (run)
            {
                if (bwt.size() + run > static_cast<size_t>(maxBlock_))
                    throw std::runtime_error("BZip2 block exceeds declared block size");
                bwt.insert(bwt.end(), static_cast<size_t>(run), mtf[0]);
                counts[mtf[0]] += static_cast<uint32_t>(run);
                run = 0;
                runBit = 0;
            }
            if (sym == alpha - 1)
                break;  // end of block
            const int idx = sym - 1;
            const uint8_t v = mtf[idx];
            for (int j = idx; j > 0; --j)
                mtf[j] = mtf[j - 1];
            mtf[0] = v;
            if (bwt.size() >= static_cast<size_t>(maxBlock_))
                throw std::runtime_error("BZip2 block exceeds declared block size");
            bwt.push_back(v);
            counts[v]++;
        }
        const uint32_t n = static_cast<uint32_t>(bwt.size());
        if (origPtr >= n)
            throw std::runtime_error("BZip2 start pointer invalid");
        // inverse BWT: next[] links each row to the row of its successor
        std::vector<uint32_t> next(n);
        uint32_t start[256];
        for (uint32_t c = 0, acc = 0; c < 256; ++c)
        {
            start[c] = acc;
            acc += counts[c];
        }
        for (uint32_t i = 0; i < n; ++i)
            next[start[bwt[i]]++] = i;
        // walk from origPtr, undoing RLE1 on the fly
        CRC32 crc;
        uint32_t row = next[origPtr];
        int last = -1, same = 0;
        for (uint32_t produced = 0; produced < n; ++produced)
        {
            const uint8_t b = bwt[row];
            row = next[row];
            if (same == 4)
            {
                for (int r = 0; r < b; ++r)
                {
                    block_.push_back(static_cast<uint8_t>(last));
                    crc.updateCRC(last);
                }
                same = 0;
                last = -1;
                continue;
            }
            if (b == last)
                same++;
            else
            {
                last = b;
                same = 1;
            }
            block_.push_back(b);
            crc.updateCRC(b);
        }
        if (static_cast<uint32_t>(crc.getCRC()) != storedCRC)
            throw std::runtime_error("BZip2 block CRC error");
        return storedCRC;
    }

    std::istream &in_;
    uint64_t acc_ = 0;
    int have_ = 0;
    bool started_ = false;
    bool done_ = false;
    bool modeChosen_ = false;  // device decoder unless BZ2MI_HOST_DECODER
    bool host_ = false;
    int maxBlock_ = 0;
    uint32_t streamCRC_ = 0;
    std::vector<uint8_t> block_;           // host decoder: the current block
    bz2mi_dctx *dctx_ = nullptr;            // device decoder
    std::vector<uint8_t> win_;              // device decoder: the input window
    std::vector<uint8_t> out_;              // device decoder: decoded bytes
    unsigned bit_ = 0;                      // window bit where decoding resumes
    size_t window_ = 0, chunk_ = 0;
    bool eof_ = false;                      // the input is read to its end
    const uint8_t *cur_ = nullptr;          // bytes being served
    size_t len_ = 0, pos_ = 0;
};

#endif
