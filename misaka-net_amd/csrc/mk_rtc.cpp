// mk_rtc.cpp -- the native tier's compiler process: compiles one generated
// module (tis_jit.h jit_module_source) for gfx950 with this ROCm install's
// hiprtc and writes the code object.
//
//   mk_rtc SOURCE_FILE CODE_OBJECT_FILE
//
// mk_exec.hip runs it as a child process: in a process that imported
// PyTorch first, PyTorch's bundled libhiprtc / libamd_comgr (the same
// sonames, an older LLVM) are what the linked hiprtc symbols resolve to,
// and they generate slower code (C4 D=256: 132 VGPRs and 325 us per launch
// against 75 VGPRs and 195 us).  Exit status 0 = code written; otherwise the
// compiler log is on stdout.
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::printf("usage: mk_rtc SOURCE_FILE CODE_OBJECT_FILE\n");
        return 2;
    }
    std::ifstream in(argv[1], std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string src = ss.str();
    if (src.empty()) {
        std::printf("mk_rtc: empty source %s\n", argv[1]);
        return 2;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "mk_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        std::printf("hiprtcCreateProgram failed\n");
        return 1;
    }
    // code object v5, as mk_exec.hip kCodeObjectVersion (why: there)
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-mcode-object-version=5"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
    size_t cs = 0;
    int rc = 0;
    if (r != HIPRTC_SUCCESS) {
        size_t ls = 0;
        (void)hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls, '\0');
        if (ls) (void)hiprtcGetProgramLog(prog, &log[0]);
        std::printf("hiprtc: %s: %s\n", hiprtcGetErrorString(r), log.substr(0, 400).c_str());
        rc = 1;
    } else if (hiprtcGetCodeSize(prog, &cs) != HIPRTC_SUCCESS || cs == 0) {
        std::printf("hiprtc produced no code\n");
        rc = 1;
    } else {
        std::vector<char> code(cs);
        (void)hiprtcGetCode(prog, code.data());
        std::ofstream out(argv[2], std::ios::binary);
        out.write(code.data(), (std::streamsize)code.size());
        if (!out) {
            std::printf("mk_rtc: cannot write %s\n", argv[2]);
            rc = 1;
        }
    }
    (void)hiprtcDestroyProgram(&prog);
    return rc;
}
