// bz2mi -- the RLE1 front end of one block, with the reference's interface
// (Stan1slav337/Bzip2-OpenCL include/BlockCompressor.hpp:35-155).
//
// Runs of 4..255 equal bytes become four copies plus a count byte (length-4);
// longer runs are cut into 255-byte pieces.  The block owns no memory: the
// caller hands in the RLE1 output buffer and the 256 "value present" flags.
// A block refuses a byte once more than blockSize-6 bytes have been flushed
// into it; its pending run is flushed by finishRLE().  The CRC covers the
// block's input bytes.
#ifndef BLOCK_COMPRESSOR_HPP
#define BLOCK_COMPRESSOR_HPP

#include <vector>

#include "CRC32.hpp"
#include "Config.hpp"

class BlockCompressor
{
public:
    BlockCompressor(unsigned char *blockPtr, bool *valuesPresentPtr, int blockSize)
        : out_(blockPtr), present_(valuesPresentPtr), limit_(blockSize - 6)
    {
    }

    bool isEmpty() { return length_ == 0 && pending_ == 0; }
    int getCRC() const { return crc_.getCRC(); }
    int getBlockLength() const { return length_; }

    // false when the block is full (the byte is not taken)
    bool write(int value)
    {
        if (length_ > limit_)
            return false;
        if (pending_ != 0 && value == current_)
        {
            if (++pending_ == 255) // a full piece is emitted at once
            {
                emit(current_, 255);
                pending_ = 0;
            }
            return true;
        }
        if (pending_ != 0)
            emit(current_, pending_);
        current_ = value;
        pending_ = 1;
        return true;
    }

    // bytes taken from data[offset, offset+length) before the block filled up
    int write(const std::vector<char> &data, int offset, int length)
    {
        int taken = 0;
        for (; taken < length; ++taken)
            if (!write(static_cast<unsigned char>(data[offset + taken])))
                break;
        return taken;
    }

    void finishRLE()
    {
        if (pending_ != 0)
        {
            emit(current_ & 0xff, pending_);
            pending_ = 0;
        }
    }

    void reset()
    {
        crc_.reset();
        length_ = 0;
        current_ = -1;
        pending_ = 0;
        for (int v = 0; v < ALPHABET_SIZE; ++v)
            present_[v] = false;
    }

private:
    void put(int v)
    {
        out_[length_++] = static_cast<unsigned char>(v);
        present_[v & 0xff] = true;
    }

    // one RLE1 piece of `run` (1..255) copies of `value`
    void emit(int value, int run)
    {
        crc_.updateCRC(value, run);
        const int copies = run < 4 ? run : 4;
        for (int i = 0; i < copies; ++i)
            put(value);
        if (run >= 4)
            put(run - 4);
    }

    unsigned char *out_;
    bool *present_;
    int limit_;
    int length_ = 0;
    int current_ = -1;
    int pending_ = 0;
    CRC32 crc_{};
};

#endif
