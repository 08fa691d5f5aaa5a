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

// OpenEXR 2 single-part scanline file, NO_COMPRESSION, HALF channels A, B, G, R (the channel list is sorted by
// name; each scanline block is one row: y, byte count, then every channel's row of halves).
namespace {
void put_le32(std::vector<uint8_t>& v, uint32_t x) {
    for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
void put_le64(std::vector<uint8_t>& v, uint64_t x) {
    for (int i = 0; i < 8; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
void attr(std::vector<uint8_t>& h, const char* name, const char* type, const std::vector<uint8_t>& value) {
    h.insert(h.end(), name, name + std::strlen(name) + 1);
    h.insert(h.end(), type, type + std::strlen(type) + 1);
    put_le32(h, (uint32_t)value.size());
    h.insert(h.end(), value.begin(), value.end());
}
}  // namespace

extern "C" int soc_write_exr(const char* path, const void* rgba16f, int32_t width, int32_t height, int32_t pitch_bytes) {
    if (!path || !rgba16f || width <= 0 || height <= 0 || pitch_bytes < width * 8)
        return set_error(SOC_E_INVALID_ARG, "soc_write_exr: bad arguments");
    std::vector<uint8_t> out;
    put_le32(out, 20000630u);   // magic 0x762f3101
    put_le32(out, 2u);          // version 2, single-part scanline
    std::vector<uint8_t> v;
    for (const char* ch : {"A", "B", "G", "R"}) {
        v.push_back((uint8_t)ch[0]);
        v.push_back(0);
        put_le32(v, 1u);                  // HALF
        v.push_back(0); v.push_back(0); v.push_back(0); v.push_back(0);   // pLinear + reserved
        put_le32(v, 1u);
        put_le32(v, 1u);                  // x / y sampling
    }
    v.push_back(0);
    attr(out, "channels", "chlist", v);
    attr(out, "compression", "compression", {0});
    v.clear();
    put_le32(v, 0); put_le32(v, 0); put_le32(v, (uint32_t)(width - 1)); put_le32(v, (uint32_t)(height - 1));
    attr(out, "dataWindow", "box2i", v);
    attr(out, "displayWindow", "box2i", v);
    attr(out, "lineOrder", "lineOrder", {0});   // INCREASING_Y
    const float one = 1.0f, zero = 0.0f;
    uint32_t bits;
    v.clear();
    std::memcpy(&bits, &one, 4);
    put_le32(v, bits);
    attr(out, "pixelAspectRatio", "float", v);
    v.clear();
    std::memcpy(&bits, &zero, 4);
    put_le32(v, bits);
    put_le32(v, bits);
    attr(out, "screenWindowCenter", "v2f", v);
    v.clear();
    std::memcpy(&bits, &one, 4);
    put_le32(v, bits);
    attr(out, "screenWindowWidth", "float", v);
    out.push_back(0);   // end of header
    const size_t row_bytes = (size_t)width * 8, block = 8 + row_bytes;
    const size_t table = out.size(), first = table + (size_t)height * 8;
    for (int y = 0; y < height; ++y) put_le64(out, first + (size_t)y * block);
    out.reserve(first + (size_t)height * block);
    static const int order[4] = {3, 2, 1, 0};   // A, B, G, R from RGBA
    for (int y = 0; y < height; ++y) {
        put_le32(out, (uint32_t)y);
        put_le32(out, (uint32_t)row_bytes);
        const uint16_t* row = reinterpret_cast<const uint16_t*>(static_cast<const uint8_t*>(rgba16f) + (size_t)y * pitch_bytes);
        for (int c : order)
            for (int x = 0; x < width; ++x) {
                const uint16_t h = row[4 * x + c];
                out.push_back((uint8_t)h);
                out.push_back((uint8_t)(h >> 8));
            }
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) return set_error(SOC_E_INVALID_ARG, "soc_write_exr: cannot open %s", path);
    const size_t w = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    if (w != out.size()) return set_error(SOC_E_INVALID_ARG, "soc_write_exr: short write to %s", path);
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
