// TEST INFRASTRUCTURE ONLY (oracle/). Never linked into the product.
//
// Prints the reference's device program text exactly as the reference's own
// host wrapper hands it to the OpenCL compiler: kernel.cpp:27-3162 builds the
// string with the R(...) stringification macro and include/kernel.hpp:7-17
// (get_opencl_c_code) post-processes it.  The Makefile compiles this file
// against the reference tree where it lies (REF=/root/reference) and writes
// the text to oracle/_ref/kernel_body.inc; nothing from the reference is copied
// into the repository.
#include <cstdio>
#include REF_KERNEL_CPP

int main() {
    std::string s = get_opencl_c_code();
    std::fwrite(s.data(), 1, s.size(), stdout);
    return 0;
}
