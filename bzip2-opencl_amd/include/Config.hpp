// bz2mi -- format and block-size constants of the bzip2 stream, under the
// names the reference's headers use (Stan1slav337/Bzip2-OpenCL
// include/Config.hpp:27-47), so code written against it keeps compiling.
#ifndef CONFIG_HPP
#define CONFIG_HPP

// ---- block sizing: the reference's -1..-9 select 10,000-byte units
// (BLOCKSIZE_DEFAULT); bz2mi also offers the bzip2-standard 100,000 unit.
static constexpr int BLOCKSIZE_DEFAULT = 10000;
static constexpr int BLOCKSIZE_BZIP2 = 100000;
static constexpr int MAX_BLOCK_SIZE = 9 * BLOCKSIZE_DEFAULT;

// ---- stream framing (48-bit magics are written as two 24-bit halves)
static constexpr int STREAM_START_MARKER_1 = 0x425a;   // "BZ"
static constexpr int STREAM_START_MARKER_2 = 0x68;     // "h"
static constexpr int BLOCK_HEADER_MARKER_1 = 0x314159; // pi
static constexpr int BLOCK_HEADER_MARKER_2 = 0x265359;
static constexpr int STREAM_END_MARKER_1 = 0x177245;   // sqrt(pi)
static constexpr int STREAM_END_MARKER_2 = 0x385090;

// ---- symbol coding
static constexpr int ALPHABET_SIZE = 256;
static constexpr int HUFFMAN_SYMBOL_RUNA = 0;
static constexpr int HUFFMAN_SYMBOL_RUNB = 1;
static constexpr int HUFFMAN_MAXIMUM_ALPHABET_SIZE = ALPHABET_SIZE + 2;
static constexpr int HUFFMAN_GROUP_RUN_LENGTH = 50;
static constexpr int HUFFMAN_MINIMUM_TABLES = 2;
static constexpr int HUFFMAN_MAXIMUM_TABLES = 6;
static constexpr int HUFFMAN_HIGH_SYMBOL_COST = 15;
static constexpr int HUFFMAN_ENCODE_MAXIMUM_CODE_LENGTH = 20;
static constexpr int HUFFMAN_DECODE_MAXIMUM_CODE_LENGTH = 23;
static constexpr int HUFFMAN_MAXIMUM_SELECTORS = MAX_BLOCK_SIZE / HUFFMAN_GROUP_RUN_LENGTH + 1;

// ---- BWT work arrays of the reference's DivSufSort (sizes only)
static constexpr int BWT_BUCKET_A_SIZE = ALPHABET_SIZE;
static constexpr int BWT_BUCKET_B_SIZE = ALPHABET_SIZE * ALPHABET_SIZE;

#endif
