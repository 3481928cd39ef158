/* TEST INFRASTRUCTURE ONLY (oracle/): command-line front end of cpu_ref.
 * usage: cpuref_cli IN OUT [-s level] [-p parallel] [-u unit] [-j threads] */
#include "cpu_ref.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s IN OUT [-s level] [-p parallel] [-u unit] [-j threads]\n", argv[0]);
        return 2;
    }
    int level = 9, p = 10, unit = 10000, threads = 1;
    for (int i = 3; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "-s")) level = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-p")) p = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-u")) unit = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-j")) threads = atoi(argv[i + 1]);
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* in = malloc(n + 1);
    if (n && fread(in, 1, n, f) != (size_t)n) {
        free(in);
        fclose(f);
        return 1;
    }
    fclose(f);
    size_t cap = cpuref_bound(n, level, unit);
    unsigned char* out = malloc(cap);
    long long r = cpuref_compress(in, n, level, p, unit, out, cap, threads);
    free(in);
    if (r < 0) {
        fprintf(stderr, "compress failed %lld\n", r);
        free(out);
        return 1;
    }
    FILE* g = fopen(argv[2], "wb");
    if (!g || fwrite(out, 1, r, g) != (size_t)r) {
        free(out);
        return 1;
    }
    fclose(g);
    free(out);
    return 0;
}
