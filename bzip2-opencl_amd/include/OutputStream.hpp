// bz2mi -- bzip2 compressing output stream with the reference's interface
// (Stan1slav337/Bzip2-OpenCL include/OutputStream.hpp:35-241), backed by the
// MI355X device compressor through the C ABI in include/bz2mi.h.
//
// Mechanism (the output bytes are the reference's):
//   * write() only appends raw bytes to a pinned host buffer; the RLE1 front
//     end, block split and CRCs (the reference's BlockCompressor::write per
//     byte, OutputStream.hpp:131-142/179-188) run on the device.  The stream is
//     handed over in units of kUnitBytes (bz2mi_unit_*): a unit's buffer holds
//     its bytes plus the next bz2mi_unit_halo() bytes, and its block chain
//     starts where the previous unit's ended.
//   * two pinned buffers alternate: while the host fills one, the device
//     compresses the unit copied from the other (RLE1, CRC, BWT, MTF run
//     asynchronously after the chain); the Huffman / assembly of a unit and
//     the write of its bytes happen when the next unit is handed over.
//   * framing on the host as in the reference: "BZh<level>" (:126-128), the
//     stream CRC chained per block (:202), end-of-stream marker and padding
//     (:163-176); units are laid out at bit offsets (no byte alignment, the
//     reference's leftover-bit carry, BitOutputStream.hpp:30-99).
// Errors: std::invalid_argument for a bad level / parallel count (:73-81),
// std::runtime_error for writes after close and for device failures (the
// reference's OpenCL wrapper exits the process instead).
#ifndef OUTPUT_STREAM_HPP
#define OUTPUT_STREAM_HPP

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "BlockCompressor.hpp"
#include "Config.hpp"
#include "bz2mi.h"

class OutputStream
{
public:
    OutputStream(std::ostream &out, int blockSizeMultiplier, int parallelBlockCnt)
        : out_(out), level_(blockSizeMultiplier), p_(parallelBlockCnt)
    {
        if (blockSizeMultiplier < 1 || blockSizeMultiplier > 9)
            throw std::invalid_argument("Invalid block size");
        if (parallelBlockCnt < 1)
            throw std::invalid_argument("Invalid parallel block count");
        int device = 0;
        if (const char *d = std::getenv("BZ2MI_DEVICE"))
            device = std::atoi(d);
        unitBytes_ = kUnitBytes;
        if (const char *u = std::getenv("BZ2MI_UNIT_BYTES"))  // tests: many small units
            unitBytes_ = static_cast<size_t>(std::atoll(u));
        ctx_ = bz2mi_create(blockSizeMultiplier, parallelBlockCnt, BLOCKSIZE_DEFAULT, device);
        if (!ctx_)
            throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
        halo_ = bz2mi_unit_halo(blockSizeMultiplier, BLOCKSIZE_DEFAULT);
        cap_ = unitBytes_ + halo_;
        for (int i = 0; i < 2; ++i)
        {
            buf_[i] = static_cast<unsigned char *>(bz2mi_host_alloc(cap_));
            unit_[i] = bz2mi_unit_create(ctx_);
            if (!buf_[i] || !unit_[i])
            {
                release();
                throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
            }
        }
        sums_.assign(static_cast<size_t>(p_) * 258, 0u);
        carried_.assign(static_cast<size_t>(p_) * 258, 0u);
        reset();
    }

    ~OutputStream()
    {
        release();
    }

    OutputStream(const OutputStream &) = delete;
    OutputStream &operator=(const OutputStream &) = delete;

    // The reference's app.cpp calls this once per input byte (app.cpp:108-114),
    // so it is one compare and one byte store: the write position is a pointer
    // bump, and a full buffer (or a closed stream: wend_ == wp_) takes the slow
    // path.  The position still goes through memory on every call (the byte
    // store may alias it), so the loop is bound by store-to-load forwarding.
    void write(int value)
    {
        unsigned char *p = wp_;
        if (p == wend_)
        {
            writeSlow(value);
            return;
        }
        *p = static_cast<unsigned char>(value);
        wp_ = p + 1;
    }

    void write(const std::vector<char> &data, int offset, int length)
    {
        if (finished_)
            throw std::runtime_error("Write beyond end of stream");
        sync();
        while (length > 0)
        {
            if (fill_ == cap_)
                handOver();
            const size_t take = std::min(static_cast<size_t>(length), cap_ - fill_);
            std::memcpy(buf_[cur_] + fill_, data.data() + offset, take);
            fill_ += take;
            offset += static_cast<int>(take);
            length -= static_cast<int>(take);
        }
        reset();
    }

    void close()
    {
        if (finished_)
            return;
        sync();
        if (fill_ == cap_)  // a full buffer is handed over as the byte writes left it
            handOver();
        finished_ = true;
        reset();
        finishPending();
        if (fill_ > 0)
        {
            // the last unit: no halo, its blocks run to the end of the stream
            startUnit(fill_, 0, BZ2MI_UNIT_ENDS_STREAM);
            finishPending();
        }
        if (!headerDone_)  // empty stream: header and trailer only
        {
            putBits(0x425a68u, 24);
            putBits(static_cast<uint32_t>('0' + level_), 8);
            headerDone_ = true;
        }
        // end-of-stream marker, stream CRC, zero padding (OutputStream.hpp:163-176)
        putBits(0x177245u, 24);
        putBits(0x385090u, 24);
        putBits(streamCRC_, 32);
        if (nbits_ & 7)
            flushByte();
        out_.flush();
    }

private:
    static constexpr size_t kUnitBytes = 64ull << 20;  // bytes per unit handed to the device

    void release()
    {
        for (int i = 0; i < 2; ++i)
        {
            if (unit_[i])
                bz2mi_unit_destroy(unit_[i]);
            if (buf_[i])
                bz2mi_host_free(buf_[i]);
            unit_[i] = nullptr;
            buf_[i] = nullptr;
        }
        if (ctx_)
            bz2mi_destroy(ctx_);
        ctx_ = nullptr;
    }

    // fill_ from the write pointer / the write pointer from fill_
    void sync()
    {
        fill_ = static_cast<size_t>(wp_ - buf_[cur_]);
    }
    void reset()
    {
        wp_ = buf_[cur_] + fill_;
        wend_ = finished_ ? wp_ : buf_[cur_] + cap_;
    }

    // write(int) found the buffer full (or the stream closed)
    void writeSlow(int value)
    {
        if (finished_)
            throw std::runtime_error("Write beyond end of stream");
        sync();
        handOver();
        reset();
        *wp_++ = static_cast<unsigned char>(value);
    }

    static void check(int rc)
    {
        if (rc != BZ2MI_OK)
            throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
    }

    // buffer full: unit [0, unitBytes_) with the halo [unitBytes_, cap_) goes to
    // the device; the halo bytes start the next buffer
    void handOver()
    {
        finishPending();
        startUnit(unitBytes_, halo_, 0);
        const int nxt = cur_ ^ 1;
        std::memcpy(buf_[nxt], buf_[cur_] + unitBytes_, halo_);
        cur_ = nxt;
        fill_ = halo_;
    }

    void startUnit(size_t own, size_t halo, int flags)
    {
        bz2mi_unit *u = unit_[cur_];
        check(bz2mi_unit_begin_host(u, buf_[cur_], own, halo, flags));
        uint64_t exit = 0, nb = 0;
        check(bz2mi_unit_chain(u, entry_, blocks_, &exit, &nb));
        entry_ = exit;
        blocks_ += nb;
        if (nb)
        {
            pending_ = u;
            pendingBlocks_ = nb;
        }
    }

    // Huffman coding and assembly of the unit handed over last, then its bytes
    void finishPending()
    {
        if (!pending_)
            return;
        bz2mi_unit *u = pending_;
        pending_ = nullptr;
        check(bz2mi_unit_sums(u, sums_.data()));
        uint64_t bits = 0;
        uint32_t share = 0;
        check(bz2mi_unit_encode(u, carried_.data(), &bits, &share));
        for (size_t i = 0; i < carried_.size(); ++i)
            carried_[i] += sums_[i];
        const uint32_t r = static_cast<uint32_t>(pendingBlocks_ & 31u);
        streamCRC_ = (r ? (streamCRC_ << r) | (streamCRC_ >> (32 - r)) : streamCRC_) ^ share;
        if (!headerDone_)
        {
            putBits(0x425a68u, 24);  // "BZh" + level (OutputStream.hpp:126-128)
            putBits(static_cast<uint32_t>('0' + level_), 8);
            headerDone_ = true;
        }
        const size_t need = static_cast<size_t>((bits + 7 + 8) / 8) + 16;
        if (stage_.size() < need)
            stage_.resize(need + need / 8);
        size_t n = 0;
        check(bz2mi_unit_assemble_host(u, nbits_, 0, 0, stage_.data(), stage_.size(), &n, nullptr));
        // the first byte shares its top (nbits_ & 7) bits with the pending byte
        if (n > 0)
        {
            stage_[0] |= partial_;
            const uint64_t end = nbits_ + bits;
            const size_t whole = static_cast<size_t>(end / 8 - nbits_ / 8);
            out_.write(reinterpret_cast<const char *>(stage_.data()), static_cast<std::streamsize>(whole));
            partial_ = (end & 7) ? stage_[whole] : 0;
            nbits_ = end;
        }
    }

    void putBits(uint32_t v, int count)
    {
        for (int k = count - 1; k >= 0; --k)
        {
            if ((v >> k) & 1u)
                partial_ |= static_cast<unsigned char>(0x80u >> (nbits_ & 7));
            ++nbits_;
            if ((nbits_ & 7) == 0)
                flushByte();
        }
    }

    void flushByte()
    {
        out_.put(static_cast<char>(partial_));
        partial_ = 0;
        nbits_ = (nbits_ + 7) & ~7ull;
    }

    std::ostream &out_;
    int level_;
    int p_;
    bz2mi_ctx *ctx_ = nullptr;
    bz2mi_unit *unit_[2] = {nullptr, nullptr};
    unsigned char *buf_[2] = {nullptr, nullptr};
    unsigned char *wp_ = nullptr, *wend_ = nullptr;  // write position, end of the buffer
    size_t unitBytes_ = 0, halo_ = 0, cap_ = 0, fill_ = 0;
    int cur_ = 0;
    bool finished_ = false, headerDone_ = false;
    uint64_t entry_ = 0, blocks_ = 0;
    bz2mi_unit *pending_ = nullptr;
    uint64_t pendingBlocks_ = 0;
    std::vector<uint32_t> sums_, carried_;
    uint32_t streamCRC_ = 0;
    uint64_t nbits_ = 0;     // stream bits so far
    unsigned char partial_ = 0;  // the byte holding bits [nbits_ & ~7, nbits_)
    std::vector<uint8_t> stage_;
};

#endif
