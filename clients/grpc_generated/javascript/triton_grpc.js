'use strict';
// Dependency-free gRPC client for inference.GRPCInferenceService on Node's
// built-in http2 module: a small protobuf wire codec for the messages the
// examples use, and gRPC length-prefixed framing over an h2c session.
// (The reference's JS example, src/grpc_generated/javascript/client.js:28-140,
// needs @grpc/grpc-js + @grpc/proto-loader; this one runs on a bare node.)

const http2 = require('http2');

// ------------------------------------------------------------ wire encoding
class Writer {
  constructor() { this.parts = []; }
  varint(v) {
    const b = [];
    let n = BigInt.asUintN(64, BigInt(v));
    while (n >= 0x80n) { b.push(Number(n & 0x7fn) | 0x80); n >>= 7n; }
    b.push(Number(n));
    this.parts.push(Buffer.from(b));
    return this;
  }
  tag(field, wire) { return this.varint(field * 8 + wire); }
  bytes(field, buf) {
    if (buf === undefined || buf === null) return this;
    const b = Buffer.isBuffer(buf) ? buf : Buffer.from(buf, 'utf8');
    this.tag(field, 2).varint(b.length);
    this.parts.push(b);
    return this;
  }
  string(field, s) { return s ? this.bytes(field, Buffer.from(s, 'utf8')) : this; }
  message(field, w) { return this.bytes(field, w.finish()); }
  bool(field, v) { return v ? this.tag(field, 0).varint(1) : this; }
  packedVarint(field, arr) {
    if (!arr || !arr.length) return this;
    const w = new Writer();
    for (const v of arr) w.varint(v);
    return this.bytes(field, w.finish());
  }
  packedFixed(field, arr, size, put) {
    if (!arr || !arr.length) return this;
    const b = Buffer.alloc(arr.length * size);
    arr.forEach((v, i) => put.call(b, v, i * size));
    return this.bytes(field, b);
  }
  finish() { return Buffer.concat(this.parts); }
}

function readVarint(buf, pos) {
  let r = 0n; let shift = 0n;
  for (;;) {
    const b = buf[pos++];
    r |= BigInt(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
    shift += 7n;
  }
  return [r, pos];
}

// Decode one message level into {field: [values]}; length-delimited values
// stay Buffers, varints become BigInt, fixed32/64 stay raw Buffers.
function fields(buf) {
  const out = {};
  let pos = 0;
  while (pos < buf.length) {
    let key; [key, pos] = readVarint(buf, pos);
    const field = Number(key >> 3n); const wire = Number(key & 7n);
    let val;
    if (wire === 0) { [val, pos] = readVarint(buf, pos); }
    else if (wire === 2) { let len; [len, pos] = readVarint(buf, pos); val = buf.subarray(pos, pos + Number(len)); pos += Number(len); }
    else if (wire === 5) { val = buf.subarray(pos, pos + 4); pos += 4; }
    else if (wire === 1) { val = buf.subarray(pos, pos + 8); pos += 8; }
    else throw new Error('unsupported wire type ' + wire);
    (out[field] = out[field] || []).push(val);
  }
  return out;
}
const str = (f, n) => (f[n] ? f[n][f[n].length - 1].toString('utf8') : '');
const flag = (f, n) => !!(f[n] && f[n][f[n].length - 1] !== 0n);
function packed(f, n) {  // repeated varint field, packed or not
  const r = [];
  for (const v of f[n] || []) {
    if (typeof v === 'bigint') { r.push(v); continue; }
    let p = 0; while (p < v.length) { let x; [x, p] = readVarint(v, p); r.push(x); }
  }
  return r;
}

// ------------------------------------------------------------- messages
const DTYPE_CONTENTS = { BOOL: 1, INT8: 2, INT16: 2, INT32: 2, INT64: 3, UINT8: 4, UINT16: 4, UINT32: 4,
                         UINT64: 5, FP32: 6, FP64: 7, BYTES: 8 };

function encodeContents(datatype, data) {
  const w = new Writer();
  const f = DTYPE_CONTENTS[datatype];
  if (f === 1) w.packedVarint(1, data.map((x) => (x ? 1 : 0)));
  else if (f === 2 || f === 3 || f === 4 || f === 5) w.packedVarint(f, data);
  else if (f === 6) w.packedFixed(6, data, 4, Buffer.prototype.writeFloatLE);
  else if (f === 7) w.packedFixed(7, data, 8, Buffer.prototype.writeDoubleLE);
  else if (f === 8) for (const s of data) w.bytes(8, Buffer.isBuffer(s) ? s : Buffer.from(String(s)));
  else throw new Error('no typed contents for ' + datatype);
  return w;
}

function encodeParameter(v) {
  const w = new Writer();
  if (typeof v === 'boolean') w.tag(1, 0).varint(v ? 1 : 0);
  else if (typeof v === 'number' && Number.isInteger(v)) w.tag(2, 0).varint(v);
  else if (typeof v === 'number') { const b = Buffer.alloc(8); b.writeDoubleLE(v); w.tag(4, 1); w.parts.push(b); }
  else w.string(3, String(v));
  return w;
}

function encodeParameters(w, field, params) {
  for (const [k, v] of Object.entries(params || {})) {
    w.message(field, new Writer().string(1, k).message(2, encodeParameter(v)));
  }
}

// request: {model_name, model_version, id, parameters, inputs:[{name, datatype, shape, data | raw}], outputs:[name]}
function encodeInferRequest(req) {
  const w = new Writer().string(1, req.model_name).string(2, req.model_version).string(3, req.id);
  encodeParameters(w, 4, req.parameters);
  const raws = [];
  for (const t of req.inputs) {
    const tw = new Writer().string(1, t.name).string(2, t.datatype).packedVarint(3, t.shape);
    encodeParameters(tw, 4, t.parameters);
    if (t.raw) raws.push(t.raw); else tw.message(5, encodeContents(t.datatype, t.data));
    w.message(5, tw);
  }
  for (const o of req.outputs || []) w.message(6, new Writer().string(1, typeof o === 'string' ? o : o.name));
  for (const r of raws) w.bytes(7, r);
  return w.finish();
}

function decodeContents(datatype, buf) {
  const f = fields(buf);
  const fid = DTYPE_CONTENTS[datatype];
  if (fid === 6 || fid === 7) {
    const size = fid === 6 ? 4 : 8; const r = [];
    for (const b of f[fid] || []) for (let p = 0; p + size <= b.length; p += size) r.push(size === 4 ? b.readFloatLE(p) : b.readDoubleLE(p));
    return r;
  }
  if (fid === 8) return (f[8] || []).map((b) => Buffer.from(b));
  const signed32 = datatype === 'INT8' || datatype === 'INT16' || datatype === 'INT32';
  return packed(f, fid).map((x) => (fid === 1 ? x !== 0n : Number(signed32 ? BigInt.asIntN(32, x) : (datatype === 'INT64' ? BigInt.asIntN(64, x) : x))));
}

const RAW_READ = { INT8: [1, 'readInt8'], UINT8: [1, 'readUInt8'], INT16: [2, 'readInt16LE'], UINT16: [2, 'readUInt16LE'],
                   INT32: [4, 'readInt32LE'], UINT32: [4, 'readUInt32LE'], FP32: [4, 'readFloatLE'], FP64: [8, 'readDoubleLE'],
                   INT64: [8, 'readBigInt64LE'], UINT64: [8, 'readBigUInt64LE'], BOOL: [1, 'readUInt8'] };

function decodeInferResponse(buf) {
  const f = fields(buf);
  const raws = f[6] || [];
  const outputs = (f[5] || []).map((ob, i) => {
    const o = fields(ob);
    const t = { name: str(o, 1), datatype: str(o, 2), shape: packed(o, 3).map(Number) };
    if (raws.length) {
      const raw = raws[i]; t.raw = Buffer.from(raw);
      const rd = RAW_READ[t.datatype];
      if (rd) { t.data = []; for (let p = 0; p + rd[0] <= raw.length; p += rd[0]) t.data.push(raw[rd[1]](p)); }
    } else if (o[5]) {
      t.data = decodeContents(t.datatype, o[5][0]);
    }
    return t;
  });
  return { model_name: str(f, 1), model_version: str(f, 2), id: str(f, 3), outputs };
}

function decodeTensorMeta(b) { const t = fields(b); return { name: str(t, 1), datatype: str(t, 2), shape: packed(t, 3).map((x) => Number(BigInt.asIntN(64, x))) }; }

// ------------------------------------------------------------- transport
class GRPCInferenceServiceClient {
  constructor(url) {
    this.session = http2.connect('http://' + url);
    this.session.on('error', () => {});
  }
  close() { this.session.close(); }

  unary(method, body) {
    return new Promise((resolve, reject) => {
      const req = this.session.request({
        ':method': 'POST', ':path': '/inference.GRPCInferenceService/' + method,
        'content-type': 'application/grpc', te: 'trailers',
      });
      const chunks = []; let status = null; let message = '';
      const onMeta = (h) => { if (h['grpc-status'] !== undefined) { status = Number(h['grpc-status']); message = decodeURIComponent(h['grpc-message'] || ''); } };
      req.on('response', onMeta);
      req.on('trailers', onMeta);
      req.on('data', (c) => chunks.push(c));
      req.on('error', reject);
      req.on('end', () => {
        if (status !== 0) { reject(new Error(`${method}: grpc-status ${status}: ${message}`)); return; }
        const all = Buffer.concat(chunks);
        if (all.length < 5) { resolve(Buffer.alloc(0)); return; }
        if (all[0] !== 0) { reject(new Error('compressed responses are not supported')); return; }
        resolve(all.subarray(5, 5 + all.readUInt32BE(1)));
      });
      const frame = Buffer.alloc(5); frame.writeUInt32BE(body.length, 1);
      req.end(Buffer.concat([frame, body]));
    });
  }

  async serverLive() { return flag(fields(await this.unary('ServerLive', Buffer.alloc(0))), 1); }
  async serverReady() { return flag(fields(await this.unary('ServerReady', Buffer.alloc(0))), 1); }
  async modelReady(name, version = '') {
    return flag(fields(await this.unary('ModelReady', new Writer().string(1, name).string(2, version).finish())), 1);
  }
  async serverMetadata() {
    const f = fields(await this.unary('ServerMetadata', Buffer.alloc(0)));
    return { name: str(f, 1), version: str(f, 2), extensions: (f[3] || []).map((b) => b.toString()) };
  }
  async modelMetadata(name, version = '') {
    const f = fields(await this.unary('ModelMetadata', new Writer().string(1, name).string(2, version).finish()));
    return { name: str(f, 1), versions: (f[2] || []).map((b) => b.toString()), platform: str(f, 3),
             inputs: (f[4] || []).map(decodeTensorMeta), outputs: (f[5] || []).map(decodeTensorMeta) };
  }
  async modelInfer(req) { return decodeInferResponse(await this.unary('ModelInfer', encodeInferRequest(req))); }
}

module.exports = { GRPCInferenceServiceClient, Writer, fields, encodeInferRequest, decodeInferResponse };
