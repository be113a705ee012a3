// Image classification client (reference src/c++/examples/image_client.cc).
//
// The reference decodes with OpenCV; the MI355X box has none, so images are
// read as binary PPM/PGM (P6/P5) and resized bilinearly here.  Everything
// else follows the reference: model metadata/config parsing (NCHW/NHWC,
// batching), NONE/INCEPTION/VGG scaling, -b batching, sync / async (-a) /
// gRPC streaming (--streaming) requests, top-k classification postprocess.
#include <dirent.h>
#include <dlfcn.h>
#include <getopt.h>
#include <hip/hip_runtime_api.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <fstream>
#include <mutex>
#include <sstream>

#include "example_util.h"
#include "grpc_client.h"
#include "http_client.h"
#include "json.h"

namespace tc = triton::client;

enum class Scale { NONE, VGG, INCEPTION };

struct ModelInfo {
  std::string input_name, output_name, datatype;
  int max_batch = 0, c = 0, h = 0, w = 0;
  bool nchw = true;
};

struct Image {
  int h = 0, w = 0, c = 0;
  std::vector<uint8_t> px;
};

static bool ReadPnm(const std::string& path, Image* img)
{
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::string magic;
  f >> magic;
  if (magic != "P6" && magic != "P5") return false;
  auto next_int = [&](int* v) {
    while (true) {
      f >> std::ws;
      if (f.peek() == '#') {
        std::string line;
        std::getline(f, line);
        continue;
      }
      f >> *v;
      return static_cast<bool>(f);
    }
  };
  int maxv;
  if (!next_int(&img->w) || !next_int(&img->h) || !next_int(&maxv) || maxv != 255) return false;
  f.get();
  img->c = magic == "P6" ? 3 : 1;
  img->px.resize(static_cast<size_t>(img->w) * img->h * img->c);
  f.read(reinterpret_cast<char*>(img->px.data()), img->px.size());
  return static_cast<size_t>(f.gcount()) == img->px.size();
}

// Resize (bilinear), convert channels, scale, lay out as NCHW/NHWC FP32.
static std::vector<uint8_t> Preprocess(const Image& img, const ModelInfo& m, Scale scale)
{
  std::vector<float> out(static_cast<size_t>(m.c) * m.h * m.w);
  for (int y = 0; y < m.h; ++y) {
    const float sy = std::max(0.f, (y + 0.5f) * img.h / m.h - 0.5f);
    const int y0 = std::min(static_cast<int>(sy), img.h - 1), y1 = std::min(y0 + 1, img.h - 1);
    const float fy = sy - y0;
    for (int x = 0; x < m.w; ++x) {
      const float sx = std::max(0.f, (x + 0.5f) * img.w / m.w - 0.5f);
      const int x0 = std::min(static_cast<int>(sx), img.w - 1), x1 = std::min(x0 + 1, img.w - 1);
      const float fx = sx - x0;
      for (int ch = 0; ch < m.c; ++ch) {
        auto at = [&](int yy, int xx) {
          if (img.c == 1) return static_cast<float>(img.px[static_cast<size_t>(yy) * img.w + xx]);
          const size_t base = (static_cast<size_t>(yy) * img.w + xx) * 3;
          if (m.c == 1)
            return (img.px[base] + img.px[base + 1] + img.px[base + 2]) / 3.0f;
          return static_cast<float>(img.px[base + ch]);
        };
        float v = (at(y0, x0) * (1 - fx) + at(y0, x1) * fx) * (1 - fy) + (at(y1, x0) * (1 - fx) + at(y1, x1) * fx) * fy;
        if (scale == Scale::INCEPTION) v = v / 127.5f - 1.0f;
        else if (scale == Scale::VGG) v -= (m.c == 3 ? (ch == 0 ? 123.f : ch == 1 ? 117.f : 104.f) : 128.f);
        const size_t idx = m.nchw ? (static_cast<size_t>(ch) * m.h + y) * m.w + x
                                  : (static_cast<size_t>(y) * m.w + x) * m.c + ch;
        out[idx] = v;
      }
    }
  }
  std::vector<uint8_t> bytes(out.size() * 4);
  memcpy(bytes.data(), out.data(), bytes.size());
  return bytes;
}

// --device-preprocess: the same resize on the host (no scaling, HWC fp32),
// then scale + HWC->CHW/HWC + FP32 for the whole batch in ONE launch of the
// framework's K6 layout_pack kernel (libtcamd_hip.so, found next to this
// build tree or via $TCAMD_HIP_LIB; hipMemcpy in and out).
typedef int (*LayoutPackFn)(const void* const*, int, int, int, void*, int, int, int, int, int, const float*,
                            const float*, int, void*);

static LayoutPackFn LoadLayoutPack()
{
  std::vector<std::string> cands;
  if (const char* env = getenv("TCAMD_HIP_LIB")) cands.push_back(env);
  char self[4096];
  const ssize_t n = readlink("/proc/self/exe", self, sizeof(self) - 1);
  if (n > 0) {
    std::string p(self, n);
    cands.push_back(p.substr(0, p.rfind('/')) + "/../../../../triton_client_amd/ops/lib/libtcamd_hip.so");
  }
  for (const auto& c : cands)
    if (void* h = dlopen(c.c_str(), RTLD_NOW | RTLD_GLOBAL))
      if (void* f = dlsym(h, "tcamd_layout_pack")) return reinterpret_cast<LayoutPackFn>(f);
  return nullptr;
}

static std::vector<std::vector<uint8_t>> PreprocessOnDevice(const std::vector<Image>& imgs, const ModelInfo& m,
                                                            Scale scale)
{
  static LayoutPackFn pack = LoadLayoutPack();
  if (!pack) {
    std::cerr << "error: --device-preprocess needs tcamd_layout_pack (libtcamd_hip.so)" << std::endl;
    exit(1);
  }
  ModelInfo hwc = m;
  hwc.nchw = false;
  const size_t per = static_cast<size_t>(m.c) * m.h * m.w;
  std::vector<float> scl(m.c, 1.f), bias(m.c, 0.f);
  for (int ch = 0; ch < m.c; ++ch) {
    if (scale == Scale::INCEPTION) {
      scl[ch] = 1.f / 127.5f;
      bias[ch] = -1.f;
    } else if (scale == Scale::VGG) {
      bias[ch] = -(m.c == 3 ? (ch == 0 ? 123.f : ch == 1 ? 117.f : 104.f) : 128.f);
    }
  }
  std::vector<std::vector<uint8_t>> out;
  for (size_t i0 = 0; i0 < imgs.size(); i0 += 64) {  // K6 takes up to 64 source pointers per launch
    const size_t cnt = std::min<size_t>(64, imgs.size() - i0);
    std::vector<uint8_t> host(cnt * per * 4);
    for (size_t i = 0; i < cnt; ++i) {
      const std::vector<uint8_t> r = Preprocess(imgs[i0 + i], hwc, Scale::NONE);
      memcpy(host.data() + i * per * 4, r.data(), r.size());
    }
    void *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, host.size()) != hipSuccess || hipMalloc(&dst, host.size()) != hipSuccess ||
        hipMemcpy(src, host.data(), host.size(), hipMemcpyHostToDevice) != hipSuccess) {
      std::cerr << "error: device buffers for --device-preprocess" << std::endl;
      exit(1);
    }
    std::vector<const void*> ptrs(cnt);
    for (size_t i = 0; i < cnt; ++i) ptrs[i] = static_cast<const uint8_t*>(src) + i * per * 4;
    const int kFp32 = 10, kNchw = 0, kNhwc = 1;
    int rc = pack(ptrs.data(), static_cast<int>(cnt), kFp32, kNhwc, dst, kFp32, m.nchw ? kNchw : kNhwc, m.c, m.h,
                  m.w, scl.data(), bias.data(), 1, nullptr);
    if (rc == 0) rc = hipMemcpy(host.data(), dst, host.size(), hipMemcpyDeviceToHost);
    (void)hipFree(src);
    (void)hipFree(dst);
    if (rc != 0) {
      std::cerr << "error: layout_pack failed (" << rc << ")" << std::endl;
      exit(1);
    }
    for (size_t i = 0; i < cnt; ++i)
      out.emplace_back(host.begin() + i * per * 4, host.begin() + (i + 1) * per * 4);
  }
  return out;
}

static void ParseDims(const std::vector<int64_t>& shape, const std::string& fmt, ModelInfo* m)
{
  std::vector<int64_t> dims(shape.begin() + (m->max_batch > 0 ? 1 : 0), shape.end());
  if (dims.size() != 3) {
    std::cerr << "error: expecting input to have 3 dims, got " << dims.size() << std::endl;
    exit(1);
  }
  m->nchw = fmt != "FORMAT_NHWC";
  if (m->nchw) {
    m->c = dims[0];
    m->h = dims[1];
    m->w = dims[2];
  } else {
    m->h = dims[0];
    m->w = dims[1];
    m->c = dims[2];
  }
}

static ModelInfo GetInfoHttp(tc::InferenceServerHttpClient* c, const std::string& model, const std::string& ver)
{
  std::string md_s, cfg_s, err;
  FAIL_IF_ERR(c->ModelMetadata(&md_s, model, ver), "unable to get model metadata");
  FAIL_IF_ERR(c->ModelConfig(&cfg_s, model, ver), "unable to get model config");
  tc::json::Value md, cfg;
  if (!tc::json::Parse(md_s, &md, &err) || !tc::json::Parse(cfg_s, &cfg, &err)) {
    std::cerr << "error: bad metadata/config json: " << err << std::endl;
    exit(1);
  }
  ModelInfo m;
  m.max_batch = cfg.Find("max_batch_size") ? static_cast<int>(cfg.Find("max_batch_size")->AsInt()) : 0;
  const auto& in = (*md.Find("inputs"))[0];
  m.input_name = in.Find("name")->AsString();
  m.datatype = in.Find("datatype")->AsString();
  m.output_name = (*md.Find("outputs"))[0].Find("name")->AsString();
  std::vector<int64_t> shape;
  for (const auto& d : in.Find("shape")->Elements()) shape.push_back(d.AsInt());
  std::string fmt = "FORMAT_NONE";
  if (const tc::json::Value* ins = cfg.Find("input"))
    if (ins->Size() && (*ins)[0].Find("format")) fmt = (*ins)[0].Find("format")->AsString();
  ParseDims(shape, fmt, &m);
  return m;
}

static ModelInfo GetInfoGrpc(tc::InferenceServerGrpcClient* c, const std::string& model, const std::string& ver)
{
  inference::ModelMetadataResponse md;
  inference::ModelConfigResponse cfg;
  FAIL_IF_ERR(c->ModelMetadata(&md, model, ver), "unable to get model metadata");
  FAIL_IF_ERR(c->ModelConfig(&cfg, model, ver), "unable to get model config");
  ModelInfo m;
  m.max_batch = cfg.config().max_batch_size();
  m.input_name = md.inputs(0).name();
  m.datatype = md.inputs(0).datatype();
  m.output_name = md.outputs(0).name();
  std::string fmt = "FORMAT_NONE";
  if (cfg.config().input_size() && cfg.config().input(0).format() == inference::ModelInput_Format_FORMAT_NHWC)
    fmt = "FORMAT_NHWC";
  ParseDims(md.inputs(0).shape(), fmt, &m);
  return m;
}

static void Postprocess(tc::InferResult* r, const std::string& out, const std::vector<std::string>& names, int topk)
{
  std::vector<std::string> classes;
  FAIL_IF_ERR(r->StringData(out, &classes), "unable to get classification output");
  if (classes.size() != names.size() * static_cast<size_t>(topk)) {
    std::cerr << "error: expected " << names.size() * topk << " classes, got " << classes.size() << std::endl;
    exit(1);
  }
  for (size_t i = 0; i < names.size(); ++i) {
    std::cout << "Image '" << names[i] << "':" << std::endl;
    for (int k = 0; k < topk; ++k) {
      std::istringstream ss(classes[i * topk + k]);
      std::string score, idx, label;
      std::getline(ss, score, ':');
      std::getline(ss, idx, ':');
      std::getline(ss, label);
      std::cout << "    " << score << " (" << idx << ") = " << label << std::endl;
    }
  }
}

int main(int argc, char** argv)
{
  bool verbose = false, async = false, streaming = false, device_pre = false;
  int batch = 1, topk = 1;
  Scale scale = Scale::NONE;
  std::string model, version, url, protocol = "http";
  static struct option long_opts[] = {{"streaming", no_argument, nullptr, 0},
                                      {"device-preprocess", no_argument, nullptr, 1},
                                      {nullptr, 0, nullptr, 0}};
  int opt;
  while ((opt = getopt_long(argc, argv, "vam:x:b:c:s:u:i:", long_opts, nullptr)) != -1) {
    switch (opt) {
      case 0: streaming = true; break;
      case 1: device_pre = true; break;
      case 'v': verbose = true; break;
      case 'a': async = true; break;
      case 'm': model = optarg; break;
      case 'x': version = optarg; break;
      case 'b': batch = std::stoi(optarg); break;
      case 'c': topk = std::stoi(optarg); break;
      case 's': {
        std::string s = optarg;
        scale = s == "INCEPTION" ? Scale::INCEPTION : s == "VGG" ? Scale::VGG : Scale::NONE;
        break;
      }
      case 'u': url = optarg; break;
      case 'i': protocol = optarg; break;
      default:
        example::Usage(argv, "\t-m <model> -x <version> -b <batch> -c <classes> -s <NONE|INCEPTION|VGG>\n"
                             "\t-i <http|grpc> -a (async) --streaming --device-preprocess <image file or dir>");
    }
  }
  for (auto& ch : protocol) ch = static_cast<char>(tolower(ch));
  if (model.empty() || optind >= argc) example::Usage(argv, "\t-m <model> is required, plus an image path");
  if (streaming && protocol != "grpc") {
    std::cerr << "Streaming is only allowed with gRPC protocol" << std::endl;
    exit(1);
  }
  const std::string path = argv[optind];
  std::vector<std::string> files;
  struct stat st;
  if (stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) {
    DIR* dir = opendir(path.c_str());
    while (dirent* e = readdir(dir))
      if (e->d_name[0] != '.') files.push_back(path + "/" + e->d_name);
    closedir(dir);
    std::sort(files.begin(), files.end());
  } else {
    files.push_back(path);
  }
  std::unique_ptr<tc::InferenceServerHttpClient> http;
  std::unique_ptr<tc::InferenceServerGrpcClient> grpcc;
  ModelInfo m;
  if (protocol == "grpc") {
    FAIL_IF_ERR(tc::InferenceServerGrpcClient::Create(&grpcc, url.empty() ? "localhost:8001" : url, verbose),
                "unable to create grpc client");
    m = GetInfoGrpc(grpcc.get(), model, version);
  } else {
    FAIL_IF_ERR(tc::InferenceServerHttpClient::Create(&http, url.empty() ? "localhost:8000" : url, verbose),
                "unable to create http client");
    m = GetInfoHttp(http.get(), model, version);
  }
  if (m.datatype != "FP32") {
    std::cerr << "error: this client sends FP32 input, model wants " << m.datatype << std::endl;
    exit(1);
  }
  if (m.max_batch == 0 && batch != 1) {
    std::cerr << "error: model does not support batching" << std::endl;
    exit(1);
  }
  std::vector<std::vector<uint8_t>> images;
  std::vector<Image> decoded;
  for (const auto& f : files) {
    Image img;
    if (!ReadPnm(f, &img)) {
      std::cerr << "error: unable to decode '" << f << "' (binary PPM/PGM expected)" << std::endl;
      exit(1);
    }
    if (device_pre) decoded.push_back(std::move(img));
    else images.push_back(Preprocess(img, m, scale));
  }
  if (device_pre) images = PreprocessOnDevice(decoded, m, scale);
  // requests of `batch` images, cycling over the list to fill the last batch
  struct Req {
    std::unique_ptr<tc::InferInput> in;
    std::unique_ptr<tc::InferRequestedOutput> out;
    std::vector<std::string> names;
  };
  std::vector<Req> reqs;
  size_t idx = 0;
  bool last = false;
  while (!last) {
    Req r;
    tc::InferInput* in;
    std::vector<int64_t> shape;
    if (m.max_batch > 0) shape.push_back(batch);
    if (m.nchw) shape.insert(shape.end(), {m.c, m.h, m.w});
    else shape.insert(shape.end(), {m.h, m.w, m.c});
    FAIL_IF_ERR(tc::InferInput::Create(&in, m.input_name, shape, "FP32"), "unable to create input");
    r.in.reset(in);
    for (int b = 0; b < batch; ++b) {
      FAIL_IF_ERR(in->AppendRaw(images[idx]), "unable to set input data");
      r.names.push_back(files[idx]);
      idx = (idx + 1) % images.size();
      if (idx == 0) last = true;
    }
    tc::InferRequestedOutput* out;
    FAIL_IF_ERR(tc::InferRequestedOutput::Create(&out, m.output_name, topk), "unable to create output");
    r.out.reset(out);
    reqs.push_back(std::move(r));
  }
  std::vector<std::unique_ptr<tc::InferResult>> results(reqs.size());
  std::mutex mu;
  std::condition_variable cv;
  size_t done = 0;
  auto on_done = [&](tc::InferResult* res) {
    std::string id;
    res->Id(&id);
    std::lock_guard<std::mutex> lk(mu);
    results[std::stoul(id)].reset(res);
    ++done;
    cv.notify_all();
  };
  if (streaming) FAIL_IF_ERR(grpcc->StartStream(on_done), "unable to start stream");
  for (size_t i = 0; i < reqs.size(); ++i) {
    tc::InferOptions options(model);
    options.model_version_ = version;
    options.request_id_ = std::to_string(i);
    std::vector<tc::InferInput*> ins = {reqs[i].in.get()};
    std::vector<const tc::InferRequestedOutput*> outs = {reqs[i].out.get()};
    if (streaming) {
      FAIL_IF_ERR(grpcc->AsyncStreamInfer(options, ins, outs), "unable to send stream request");
    } else if (async) {
      FAIL_IF_ERR(grpcc ? grpcc->AsyncInfer(on_done, options, ins, outs) : http->AsyncInfer(on_done, options, ins, outs),
                  "unable to send async request");
    } else {
      tc::InferResult* res;
      FAIL_IF_ERR(grpcc ? grpcc->Infer(&res, options, ins, outs) : http->Infer(&res, options, ins, outs),
                  "unable to run model");
      on_done(res);
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return done == reqs.size(); })) {
      std::cerr << "error: timed out waiting for results" << std::endl;
      exit(1);
    }
  }
  if (streaming) grpcc->StopStream();
  for (size_t i = 0; i < reqs.size(); ++i) {
    FAIL_IF_ERR(results[i]->RequestStatus(), "inference failed");
    std::cout << "Request " << i << ", batch size " << batch << std::endl;
    Postprocess(results[i].get(), m.output_name, reqs[i].names, topk);
  }
  std::cout << "PASS" << std::endl;
  return 0;
}
