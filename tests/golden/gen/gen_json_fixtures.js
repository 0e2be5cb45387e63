// JSON.parse / JSON.stringify forms for the engine's ContentJSON / Embed / Format check (yc_parse.h json_check).
// TEST INFRASTRUCTURE ONLY: seeded JSON values from a small vocabulary (numbers at the edges of
// Number::toString's forms, escapes, surrogates, array-index keys), stringified, then mutated by one
// inserted / replaced character; each recorded with what Node's JSON does with it.
// Usage: node gen_json_fixtures.js <out_dir>  ->  <out_dir>/json_forms.json
// JSON.parse / JSON.stringify oracle for the json_check probe (test only)
function rnd(seed){let a=seed;return()=>{a|=0;a=a+0x6D2B79F5|0;let t=Math.imul(a^a>>>15,1|a);t=t+Math.imul(t^t>>>7,61|t)^t;return((t^t>>>14)>>>0)/4294967296;}}
const r=rnd(7);
const pick=a=>a[Math.floor(r()*a.length)];
function val(d){const x=r();
 if(d>3||x<0.35){return pick([0,1,-1,1.5,-0.25,1e21,1e-7,123456789012345,1234567890123456,0.1,0.000001,1e300,5e-324,2e-308,-0,true,false,null,"a","é","\n","\u2028","\ud83d\ude00","x\"y","\\","/","\u0001","\u007f",""]);}
 if(x<0.6){const n=Math.floor(r()*4);const a=[];for(let i=0;i<n;i++)a.push(val(d+1));return a;}
 const n=Math.floor(r()*4);const o={};for(let i=0;i<n;i++)o[pick(["a","b","0","12","__proto__","k","é"])]=val(d+1);return o;}
const out=new Set();
const hand=['1','01','1.0','1e5','1E5','1e+5','-0','0','0.0','"\\u0041"','"\\/"','"\\u001f"','"\\u001F"','"\\b"','"\\u0008"','"\\ud800"','"\\ud800\\udc00"','"\\udc00"',' 1','1 ','[1, 2]','[1,2]','{"a":1,"a":2}','{"b":1,"a":2}','{"1":1,"a":2}','{"a":1,"1":2}','[]','{}','[ ]','nul','tru','"abc','"a\tb"','1.','.5','-','1e','1e+','00','-01','1e21','1e+21','100000000000000000000','1000000000000000000000','0.000001','0.0000001','1e-7','123456789012345678','12345678901234567','1234567890123456','999999999999999','9007199254740993','1.7976931348623157e+308','1e309','5e-324','[[[[1]]]]','{"a":{"b":[1,{"c":null}]}}','"\u2028"','true','false','null','undefined','"\\u00e9"','"é"','[1,]','{"a":1,}','{"a"1}','{a:1}',"'a'",'"\\x41"','-1.5e-10','1.5e-7','0.00001','2.5e+25','1e-6','1.25','12.50','-12.5'];
for(const h of hand) out.add(h);
for(let i=0;i<4000;i++){let s=JSON.stringify(val(0));
 if(r()<0.5){const k=Math.floor(r()*(s.length+1));const ins=pick([' ','0','.','e','-','"','\\','1',',',']','}','[','{',':','\t','E','+']);
  if(r()<0.5) s=s.slice(0,k)+ins+s.slice(k); else s=s.slice(0,k)+ins+s.slice(k+1);}
 out.add(s);}
const res=[];
for(const s of out){ if(s.includes('\n') || Buffer.from(Buffer.from(s,'utf8').toString('utf8'),'utf8').toString('utf8')!==s || Buffer.from(s,'utf8').toString('utf8')!==s) continue; let c; try{const v=JSON.parse(s); c=JSON.stringify(v)===s?0:2;}catch(e){c=1;} res.push(c+' '+Buffer.from(s,'utf8').toString('hex'));}
const outDir = process.argv[2] || require('path').join(__dirname, '..');
require('fs').writeFileSync(require('path').join(outDir, 'json_forms.json'), JSON.stringify({ node: process.version, note: 'want: 0 JSON.stringify(JSON.parse(s)) === s, 1 JSON.parse throws, 2 otherwise; s as UTF-8 hex', cases: res.map((x) => x.split(' ')).map(([w, h]) => [+w, h]) }));
console.log(res.length);
