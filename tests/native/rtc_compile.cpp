// rtc_compile.cpp -- TEST TOOL (not part of the product): compiles one
// generated module (tis_jit.h jit_module_source / the session module) for
// gfx950 with this ROCm install's hiprtc, in a process of its own that never
// loads PyTorch, and writes the code object.
//
//   rtc_compile SOURCE_FILE CODE_OBJECT_FILE
//
// Tests use it (built by tests/schedcheck.py rtc_tool) to check that the
// generated sources compile without a GPU, and that the executor's in-process
// namespace compiler (mk_exec.hip ns_rtc) yields byte-identical code objects.
// Until round 5 the product ran this as a child process of a GPU-initialised
// process (MK_HIPRTC=helper); that path was removed.  Exit
// status 0 = code written; otherwise the compiler log is on stdout.
#include <hip/hiprtc.h>

#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char **argv)
{
    if (argc != 3) {
        std::printf("usage: rtc_compile SOURCE_FILE CODE_OBJECT_FILE\n");
        return 2;
    }
    std::ifstream in(argv[1], std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string src = ss.str();
    if (src.empty()) {
        std::printf("rtc_compile: empty source %s\n", argv[1]);
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
            std::printf("rtc_compile: cannot write %s\n", argv[2]);
            rc = 1;
        }
    }
    (void)hiprtcDestroyProgram(&prog);
    return rc;
}
