// Where the end-to-end time of the drop-in app goes (bench.py --mode e2e).
// The reference's app.cpp (app.cpp:104-116) reads the file in 128 KB chunks
// and calls OutputStream::write(int) once per byte; this program times the
// same pieces one at a time in one process, on the mirror OutputStream:
//   init      OutputStream construction (HIP init, device context, pinned buffers)
//   read      the file read in 128 KB chunks (page cache), nothing else
//   loop      the per-byte write(int) loop over bytes already in memory into a
//             host-only sink with the mirror's write(int) (pointer bump),
//             no device: the loop's own bound
//   compress  the per-byte loop from memory into the real OutputStream + close()
//             (device units overlapped with the loop, output file written)
// Usage: e2e_parts <file> <level> <parallel> <out>; prints one JSON object.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <vector>

#include "OutputStream.hpp"

namespace {

using Clock = std::chrono::steady_clock;

double since(Clock::time_point t0)
{
    return std::chrono::duration<double>(Clock::now() - t0).count();
}

// the hot path of OutputStream::write(int) without the device behind it
struct HostSink
{
    explicit HostSink(size_t cap) : ring(cap), wp(ring.data()), wend(ring.data() + cap) {}
    __attribute__((noinline)) void slow(int v)
    {
        ++wraps;
        wp = ring.data();
        *wp++ = static_cast<unsigned char>(v);
    }
    void write(int value)
    {
        unsigned char *p = wp;
        if (p == wend)
        {
            slow(value);
            return;
        }
        *p = static_cast<unsigned char>(value);
        wp = p + 1;
    }
    std::vector<unsigned char> ring;
    unsigned char *wp, *wend;
    size_t wraps = 0;
};

// app.cpp's loop shape: 128 KB chunks, one write(int) per byte
template <class Sink>
void feed(Sink &s, const std::vector<char> &data)
{
    const size_t chunk = 131072;
    std::vector<char> buffer(chunk);
    for (size_t off = 0; off < data.size(); off += chunk)
    {
        const size_t n = std::min(chunk, data.size() - off);
        std::memcpy(buffer.data(), data.data() + off, n);
        for (int i = 0; i < static_cast<int>(n); ++i)
            s.write(buffer[i]);
    }
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc < 5)
    {
        std::fprintf(stderr, "usage: e2e_parts <file> <level> <parallel> <out>\n");
        return 2;
    }
    const int level = std::atoi(argv[2]), par = std::atoi(argv[3]);
    // read
    auto t0 = Clock::now();
    std::vector<char> data;
    {
        std::ifstream in(argv[1], std::ios::binary);
        std::vector<char> buffer(131072);
        while (in)
        {
            in.read(buffer.data(), static_cast<std::streamsize>(buffer.size()));
            data.insert(data.end(), buffer.data(), buffer.data() + in.gcount());
        }
    }
    const double t_read = since(t0);
    // loop (host only)
    HostSink sink(64u << 20);
    t0 = Clock::now();
    feed(sink, data);
    const double t_loop = since(t0);
    // init + compress
    std::ofstream out(argv[4], std::ios::binary);
    t0 = Clock::now();
    OutputStream bz(out, level, par);
    const double t_init = since(t0);
    t0 = Clock::now();
    feed(bz, data);
    bz.close();
    out.flush();
    const double t_comp = since(t0);
    const double mb = static_cast<double>(data.size()) / 1e6;
    std::printf("{\"bytes\": %zu, \"init_s\": %.4f, \"read_s\": %.4f, \"read_MBps\": %.1f, \"loop_s\": %.4f, "
                "\"loop_MBps\": %.1f, \"compress_s\": %.4f, \"compress_MBps\": %.1f, \"sink_wraps\": %zu}\n",
                data.size(), t_init, t_read, mb / t_read, t_loop, mb / t_loop, t_comp, mb / t_comp, sink.wraps);
    return 0;
}
