// bz2mi -- bzip2 compressing output stream with the reference's interface
// (Stan1slav337/Bzip2-OpenCL include/OutputStream.hpp:35-241), backed by the
// MI355X device compressor through the C ABI in include/bz2mi.h.
//
// Differences in mechanism, not in output:
//   * blocks are handed to the device in batches of many blocks instead of
//     `p` at a time (the reference's closeBlocks, :190-240).  The Huffman seed
//     carry-over still follows block index mod p (its never-cleared per-slot
//     frequency array), so the bytes are identical for every batch size;
//   * packed bits instead of bool-per-bit buffers, stitched on the device.
// Errors: std::invalid_argument for a bad level / parallel count (:73-81),
// std::runtime_error for writes after close and for device failures (the
// reference's OpenCL wrapper exits the process instead).
#ifndef OUTPUT_STREAM_HPP
#define OUTPUT_STREAM_HPP

#include <cstdlib>
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
        : out_(out), blockSize_(BLOCKSIZE_DEFAULT * blockSizeMultiplier)
    {
        if (blockSizeMultiplier < 1 || blockSizeMultiplier > 9)
            throw std::invalid_argument("Invalid block size");
        if (parallelBlockCnt < 1)
            throw std::invalid_argument("Invalid parallel block count");
        int device = 0;
        if (const char *d = std::getenv("BZ2MI_DEVICE"))
            device = std::atoi(d);
        ctx_ = bz2mi_create(blockSizeMultiplier, parallelBlockCnt, BLOCKSIZE_DEFAULT, device);
        if (!ctx_)
            throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
        stride_ = static_cast<size_t>(blockSize_) + 16;
        batch_ = kBatchBlocks;
        blocks_.resize(batch_ * stride_);
        present_.resize(static_cast<size_t>(batch_) * ALPHABET_SIZE);
        lens_.resize(batch_);
        crcs_.resize(batch_);
        for (int i = 0; i < batch_; ++i)
            compressors_.emplace_back(blocks_.data() + i * stride_,
                                      reinterpret_cast<bool *>(present_.data()) + i * ALPHABET_SIZE, blockSize_);
        staging_.resize(bz2mi_compress_bound(static_cast<size_t>(batch_) * blockSize_, blockSizeMultiplier,
                                             BLOCKSIZE_DEFAULT));
    }

    ~OutputStream()
    {
        bz2mi_destroy(ctx_);
    }

    OutputStream(const OutputStream &) = delete;
    OutputStream &operator=(const OutputStream &) = delete;

    void write(int value)
    {
        if (finished_)
            throw std::runtime_error("Write beyond end of stream");
        if (!compressors_[current_].write(value & 0xff))
        {
            nextCompressor();
            compressors_[current_].write(value & 0xff);
        }
    }

    void write(const std::vector<char> &data, int offset, int length)
    {
        if (finished_)
            throw std::runtime_error("Write beyond end of stream");
        while (length > 0)
        {
            const int taken = compressors_[current_].write(data, offset, length);
            if (taken < length)
                nextCompressor();
            offset += taken;
            length -= taken;
        }
    }

    void close()
    {
        if (finished_)
            return;
        finished_ = true;
        flushBlocks(current_ + (compressors_[current_].isEmpty() ? 0 : 1));
        size_t n = 0;
        check(bz2mi_finish(ctx_, staging_.data(), staging_.size(), &n));
        out_.write(reinterpret_cast<const char *>(staging_.data()), static_cast<std::streamsize>(n));
        out_.flush();
    }

private:
    static constexpr int kBatchBlocks = 1024;  // blocks per device call

    void nextCompressor()
    {
        if (++current_ == batch_)
        {
            flushBlocks(batch_);
            current_ = 0;
        }
    }

    // close `count` filled blocks and hand them to the device
    void flushBlocks(int count)
    {
        for (int i = 0; i < count; ++i)
        {
            BlockCompressor &bc = compressors_[i];
            bc.finishRLE();
            lens_[i] = static_cast<uint32_t>(bc.getBlockLength());
            crcs_[i] = static_cast<uint32_t>(bc.getCRC());
        }
        if (count > 0)
        {
            size_t n = 0;
            check(bz2mi_compress_rle1(ctx_, blocks_.data(), stride_, lens_.data(), crcs_.data(),
                                      static_cast<uint32_t>(count), staging_.data(), staging_.size(), &n));
            out_.write(reinterpret_cast<const char *>(staging_.data()), static_cast<std::streamsize>(n));
        }
        for (int i = 0; i < count; ++i)
            compressors_[i].reset();
    }

    static void check(int rc)
    {
        if (rc != BZ2MI_OK)
            throw std::runtime_error(std::string("bz2mi: ") + bz2mi_last_error());
    }

    std::ostream &out_;
    int blockSize_;
    bz2mi_ctx *ctx_ = nullptr;
    bool finished_ = false;
    int current_ = 0;
    int batch_ = 0;
    size_t stride_ = 0;
    std::vector<unsigned char> blocks_;
    std::vector<unsigned char> present_;
    std::vector<uint32_t> lens_, crcs_;
    std::vector<BlockCompressor> compressors_;
    std::vector<uint8_t> staging_;
};

#endif
