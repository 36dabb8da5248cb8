"""Repository style check (the role of the reference's ``make check``:
jsl + jsstyle + bashstyle, tools/mk/Makefile.targ:194-213).  No third-party
linters are installed here, so this is a small self-contained checker:

  Python  compiles; lines <= 79 columns; no tabs / trailing whitespace;
          imports never used in the module (``# noqa`` exempts a line).
  C++/HIP lines <= 100 columns; no tabs / trailing whitespace.
  shell   ``bash -n`` parses; lines <= 100 columns.

Exit status 1 with one ``file:line: message`` per finding."""

import ast
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {'.git', 'build', '__pycache__', 'gpurun_out', '.pytest_cache',
             '.hypothesis', 'profiles', '.claude'}


def files():
    for d, dirs, fs in os.walk(ROOT):
        dirs[:] = [x for x in dirs if x not in SKIP_DIRS]
        for f in fs:
            yield os.path.join(d, f)


def text_checks(path, limit, out):
    with open(path, encoding='utf-8', errors='replace') as fh:
        for i, line in enumerate(fh, 1):
            line = line.rstrip('\n')
            if '\t' in line:
                out.append('%s:%d: tab character' % (path, i))
            if line != line.rstrip():
                out.append('%s:%d: trailing whitespace' % (path, i))
            if len(line) > limit and 'noqa' not in line and \
                    'http' not in line:
                out.append('%s:%d: line too long (%d > %d)' %
                           (path, i, len(line), limit))


def unused_imports(path, src, out):
    tree = ast.parse(src, path)
    lines = src.splitlines()
    imported = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if 'noqa' in lines[node.lineno - 1]:
                continue
            for a in node.names:
                name = (a.asname or a.name).split('.')[0]
                if name != '*':
                    imported[name] = node.lineno
    used = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            pass
    # names referenced as the root of attribute chains are ast.Name too;
    # names re-exported through __all__ count as used
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Name) and t.id == '__all__'
                for t in node.targets):
            for elt in getattr(node.value, 'elts', []):
                if isinstance(elt, ast.Constant):
                    used.add(elt.value)
    if os.path.basename(path) == '__init__.py':
        return
    for name, ln in sorted(imported.items(), key=lambda x: x[1]):
        if name not in used:
            out.append('%s:%d: %r imported but unused' % (path, ln, name))


def main():
    out = []
    for path in files():
        rel = os.path.relpath(path, ROOT)
        if path.endswith('.py'):
            src = open(path, encoding='utf-8').read()
            try:
                compile(src, path, 'exec')
            except SyntaxError as e:
                out.append('%s:%d: syntax error: %s' % (rel, e.lineno, e.msg))
                continue
            text_checks(path, 79, out)
            unused_imports(path, src, out)
        elif path.endswith(('.hip', '.h', '.cpp', '.cc')):
            text_checks(path, 100, out)
        elif path.endswith('.sh'):
            text_checks(path, 100, out)
            r = subprocess.run(['bash', '-n', path], capture_output=True,
                               text=True)
            if r.returncode != 0:
                out.append('%s:1: bash -n: %s' % (rel, r.stderr.strip()))
    for line in out:
        print(os.path.relpath(line, ROOT) if line.startswith(ROOT) else line)
    return 1 if out else 0


if __name__ == '__main__':
    sys.exit(main())
