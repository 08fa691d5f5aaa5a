// output.cpp — headless output + observability: framebuffer readback, a PNG writer
// for the RGBA8 swapchain image, and the per-frame GPU-metric record of the reference's "GPU Metric"
// window (renderer.cpp:769-806) as one JSON object.
//
// The reference presents the tone-mapped image to a swapchain (tone_mapping.inl:172-176) and shows the
// per-task GPU times summed into 12 named groups (renderer.cpp:558-588) in ImGui. Headless, the image
// goes to a host buffer / PNG file and the metrics to a JSON line per frame.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "soc_internal.hpp"

using namespace soc;

namespace {

uint32_t crc_table[256];
bool crc_ready = false;

void crc_init() {
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}

uint32_t crc32(uint32_t crc, const uint8_t* p, size_t n) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = crc_table[(crc ^ p[i]) & 255u] ^ (crc >> 8);
    return ~crc;
}

void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16)); v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}

void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put_be32(out, crc32(0, out.data() + start, out.size() - start));
}

}  // namespace

// PNG (8-bit RGBA, no interlace) with an uncompressed ("stored") zlib stream: no external library.
extern "C" int soc_write_png(const char* path, const void* rgba8, int32_t width, int32_t height, int32_t pitch_bytes) {
    if (!path || !rgba8 || width <= 0 || height <= 0 || pitch_bytes < width * 4)
        return set_error(SOC_E_INVALID_ARG, "soc_write_png: bad arguments");
    if (!crc_ready) crc_init();
    std::vector<uint8_t> raw;
    raw.reserve((size_t)height * (width * 4 + 1));
    for (int y = 0; y < height; ++y) {
        raw.push_back(0);   // filter: none
        const uint8_t* row = static_cast<const uint8_t*>(rgba8) + (size_t)y * pitch_bytes;
        raw.insert(raw.end(), row, row + (size_t)width * 4);
    }
    std::vector<uint8_t> z;
    z.reserve(raw.size() + raw.size() / 65535 * 5 + 16);
    z.push_back(0x78); z.push_back(0x01);
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;   // Adler-32
    for (uint8_t c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width);
    put_be32(ihdr, (uint32_t)height);
    ihdr.push_back(8); ihdr.push_back(6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);   // 8-bit RGBA
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    FILE* f = std::fopen(path, "wb");
    if (!f) return set_error(SOC_E_INVALID_ARG, "soc_write_png: cannot open %s", path);
    const size_t w = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    if (w != out.size()) return set_error(SOC_E_INVALID_ARG, "soc_write_png: short write to %s", path);
    return SOC_OK;
}

// Device image -> host rows (stream-ordered; the caller synchronises before reading `host`).
extern "C" int soc_read_image(soc_img image, void* host, int32_t host_pitch_bytes, soc_stream stream) {
    int rc = check_img(image, 0, "soc_read_image", "image");
    if (rc) return rc;
    const int row = image.width * bytes_per_pixel(image.format);
    if (!host || host_pitch_bytes < row) return set_error(SOC_E_INVALID_ARG, "soc_read_image: bad host buffer");
    if (hipMemcpy2DAsync(host, host_pitch_bytes, image.data, image.pitch_bytes, row, image.height, hipMemcpyDeviceToHost,
                         hs(stream)) != hipSuccess)
        return set_error(SOC_E_HIP, "soc_read_image: copy failed");
    return SOC_OK;
}
