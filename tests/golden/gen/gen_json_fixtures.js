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
// re-serialisation cases (round 6: the engine rewrites non-canonical values instead of refusing them):
// long and edge numbers, deep nesting, duplicate / index / escaped keys, escapes of every kind
const hand2=['0.30000000000000004','0.1e1','100e-2','1e400','-1e400','1e-400','-1e-400','2.4703282292062327e-324','2.4703282292062328e-324',
 '1.7976931348623158e308','1.7976931348623159e308','9007199254740993','9007199254740995','123456789012345678901234567890','0.'+'0'.repeat(300)+'1',
 '1'+'0'.repeat(400),'3.'+'1'.repeat(900),'4.9406564584124654e-324','2.2250738585072011e-308','2.2250738585072014e-308','1.00000000000000011102230246251565404236316680908203125',
 '1.00000000000000011102230246251565404236316680908203124','1.00000000000000011102230246251565404236316680908203126','5e-7','-5E+22','1e21','123e19','0.000001234','1.5e-6',
 '['.repeat(100)+']'.repeat(100),'['.repeat(70)+'1'+']'.repeat(70),'{"a":'.repeat(80)+'1'+'}'.repeat(80),'['.repeat(40)+'{"x": [1, 2.50, "\\u0041"]}'+']'.repeat(40),
 '{"b":1,"a":2,"b":3}','{"2":1,"1":2,"a":3,"0":4}','{"a":1,"\\u0061":2}','{"4294967294":1,"4294967295":2,"01":3,"1":4}','{"__proto__":1,"a":{"__proto__":[]}}',
 '{ "k" : [ 1 , { "j" : null } ] , "k" : true }','"\\u00e9\\u20ac\\ud83d\\ude00"','"\\uD83D\\uDE00"','"\\ud83d"','"\\ude00\\ud83d"','"\\/\\"\\\\"','"\\u0000\\u001F\\u007f\\u2028"',
 '"\\b\\f\\n\\r\\t\\u0008\\u000c"','[1.0,2.50,-0.0,1E2,1e+2,0.5e-0]',' { } ','\t[\r\n]\n','{"a":[],"b":{},"a":{}}','{"1":{"1":1,"0":0},"0":[{"b":1,"a":0}]}'];
for(const h of hand2) out.add(h);
{ const r2=rnd(11); const pick2=a=>a[Math.floor(r2()*a.length)]; for(let i=0;i<3000;i++){ const x=r2(); let s;
  if(x<0.4){ const b=new Float64Array(1); const u=new Uint32Array(b.buffer); u[0]=(r2()*4294967296)>>>0; u[1]=(r2()*2146435072)>>>0; const v=b[0];
    s=[v.toPrecision(17),v.toPrecision(21),v.toExponential(19),String(v),v.toPrecision(1+Math.floor(r2()*20))][Math.floor(r2()*5)]; }
  else if(x<0.7){ const nd=1+Math.floor(r2()*40); s=''; for(let k=0;k<nd;k++) s+=Math.floor(r2()*10); s=s.replace(/^0+(?=\d)/,''); if(r2()<0.5&&s.length>1) s=s[0]+'.'+s.slice(1); if(r2()<0.6) s+='e'+(r2()<0.5?'-':'+')+Math.floor(r2()*330); }
  else { const parts=[]; const n=1+Math.floor(r2()*4); for(let k=0;k<n;k++) parts.push(pick2(['"a"','"b"','"0"','"1"','"10"','"\\u0062"'])+': '+pick2(['1','1.50','"x"','[ ]','{"a":1,"a":2}','null','2e3'])); s='{'+parts.join(' ,')+'}'; }
  if(r2()<0.3 && s[0]!=='{') s='-'+s; out.add(s); } }
for(let i=0;i<4000;i++){let s=JSON.stringify(val(0));
 if(r()<0.5){const k=Math.floor(r()*(s.length+1));const ins=pick([' ','0','.','e','-','"','\\','1',',',']','}','[','{',':','\t','E','+']);
  if(r()<0.5) s=s.slice(0,k)+ins+s.slice(k); else s=s.slice(0,k)+ins+s.slice(k+1);}
 out.add(s);}
const res=[];
for(const s of out){ if(s.includes('\n') || Buffer.from(Buffer.from(s,'utf8').toString('utf8'),'utf8').toString('utf8')!==s || Buffer.from(s,'utf8').toString('utf8')!==s) continue; let c, canon=''; try{const v=JSON.parse(s); const t=JSON.stringify(v); c=t===s?0:2; canon=Buffer.from(t,'utf8').toString('hex');}catch(e){c=1;} res.push(c+' '+Buffer.from(s,'utf8').toString('hex')+' '+canon);}
const outDir = process.argv[2] || require('path').join(__dirname, '..');
require('fs').writeFileSync(require('path').join(outDir, 'json_forms.json'), JSON.stringify({ node: process.version, note: 'want: 0 JSON.stringify(JSON.parse(s)) === s, 1 JSON.parse throws, 2 otherwise; s as UTF-8 hex; then JSON.stringify(JSON.parse(s)) as UTF-8 hex (empty when it throws)', cases: res.map((x) => x.split(' ')).map(([w, h, c]) => [+w, h, c || '']) }));
console.log(res.length);
