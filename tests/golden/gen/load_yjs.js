// Fixture-generation helper (TEST INFRASTRUCTURE ONLY — never part of the product). Also used by
// scripts/yjs_baseline.js, bench.py's CPU-baseline leg, which times the machine's OWN installed
// Yjs copy (the same image on the GPU box); no Yjs code is shipped with this repository.
//
// Loads the Yjs 13.5.16 + lib0 0.2.42 bundle that ships inside this container's JupyterLab
// static assets (SURVEY.md §4.1, §8(c)). No Yjs code lives in this repository: this file is a
// ~20-line webpack-runtime stand-in that evaluates the three chunks in place and returns the
// module that exports the public Yjs API (module id 73502).
'use strict';
const fs = require('fs');

const STATIC = '/opt/conda/share/jupyter/lab/static/';
const CHUNKS = [
  '8086.1dfabaac37d971e2cc4c.js', // lib0 0.2.42
  '1057.1a1aee857cdaddbae1d3.js', // lib0 helpers
  '3502.fbe0c610be82ba1360db.js', // yjs 13.5.16
];

function loadYjs() {
  global.self = global;
  if (!global.crypto) {
    global.crypto = { getRandomValues: (b) => require('crypto').randomFillSync(b) };
  }
  const modules = {};
  global.webpackChunk_jupyterlab_application_top = {
    push: ([, m]) => Object.assign(modules, m),
  };
  for (const f of CHUNKS) {
    // eslint-disable-next-line no-eval
    eval(fs.readFileSync(STATIC + f, "utf8"));
  }
  const cache = {};
  const req = (id) => {
    if (cache[id]) return cache[id].exports;
    const m = { exports: {} };
    cache[id] = m;
    if (!modules[id]) throw new Error('webpack module missing: ' + id);
    modules[id](m, m.exports, req);
    return m.exports;
  };
  req.r = (e) => Object.defineProperty(e, '__esModule', { value: true });
  req.d = (e, d) => {
    for (const k in d) {
      if (!Object.prototype.hasOwnProperty.call(e, k)) {
        Object.defineProperty(e, k, { enumerable: true, get: d[k] });
      }
    }
  };
  req.o = (o, p) => Object.prototype.hasOwnProperty.call(o, p);
  req.g = global;
  req.n = (m) => {
    const g = m && m.__esModule ? () => m.default : () => m;
    req.d(g, { a: g });
    return g;
  };
  return req(73502);
}

module.exports = { loadYjs };
