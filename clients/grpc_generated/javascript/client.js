'use strict';
// add/sub on "simple" over gRPC from Node, with typed int_contents inputs and
// raw little-endian inputs (reference src/grpc_generated/javascript/client.js).
//   node client.js [host:port]
const { GRPCInferenceServiceClient } = require('./triton_grpc');

async function main() {
  const url = process.argv[2] || 'localhost:8001';
  const client = new GRPCInferenceServiceClient(url);
  try {
    console.log('server live:', await client.serverLive());
    console.log('server ready:', await client.serverReady());
    console.log('model ready:', await client.modelReady('simple'));
    const md = await client.modelMetadata('simple');
    console.log('model metadata:', JSON.stringify(md));
    const a = Array.from({ length: 16 }, (_, i) => i);
    const b = Array(16).fill(1);
    // typed contents (int_contents)
    let r = await client.modelInfer({
      model_name: 'simple', id: 'js-typed',
      inputs: [{ name: 'INPUT0', datatype: 'INT32', shape: [1, 16], data: a },
               { name: 'INPUT1', datatype: 'INT32', shape: [1, 16], data: b }],
      outputs: ['OUTPUT0', 'OUTPUT1'],
    });
    check(r, a, b);
    // raw_input_contents
    const raw = (arr) => { const buf = Buffer.alloc(arr.length * 4); arr.forEach((v, i) => buf.writeInt32LE(v, i * 4)); return buf; };
    r = await client.modelInfer({
      model_name: 'simple', id: 'js-raw',
      inputs: [{ name: 'INPUT0', datatype: 'INT32', shape: [1, 16], raw: raw(a) },
               { name: 'INPUT1', datatype: 'INT32', shape: [1, 16], raw: raw(b) }],
      outputs: ['OUTPUT0', 'OUTPUT1'],
    });
    check(r, a, b);
    console.log('PASS: js grpc client');
  } finally {
    client.close();
  }
}

function check(r, a, b) {
  const sum = r.outputs.find((o) => o.name === 'OUTPUT0').data;
  const diff = r.outputs.find((o) => o.name === 'OUTPUT1').data;
  for (let i = 0; i < 16; i++) {
    console.log(`${a[i]} + ${b[i]} = ${sum[i]}; ${a[i]} - ${b[i]} = ${diff[i]}`);
    if (sum[i] !== a[i] + b[i] || diff[i] !== a[i] - b[i]) throw new Error('incorrect result');
  }
}

main().catch((e) => { console.error('error:', e.message); process.exit(1); });
