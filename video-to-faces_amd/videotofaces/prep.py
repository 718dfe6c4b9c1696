"""Argument validation and input listing of the public API (drop-in for
src/videotofaces/prep.py): same accepted values, same ERROR messages, same return-None
behaviour.  Control plane, not the hot path; kept so video_to_faces() behaves identically."""
import os
import os.path as osp

IMG_EXTENSIONS = ('.jpg', '.jpeg', '.png', '.ppm', '.bmp', '.pgm', '.tif', '.tiff', '.webp')
LIVE_DET, LIVE_ENC = ('default', 'yolo', 'mtcnn'), ('default', 'facenet_vgg', 'facenet_casia')
ANIME_DET, ANIME_ENC = ('default', 'rcnn'), ('default', 'vit_b', 'vit_l')


def get_img_paths(target_dir):
    if not osp.isdir(target_dir):
        return []
    return sorted(e.path for e in os.scandir(target_dir) if e.is_file() and e.name.lower().endswith(IMG_EXTENSIONS))


def _one_of(val, name, allowed):
    if val in allowed:
        return True
    print('ERROR: unknown %s. Available options are %s' % (name, ', '.join('"%s"' % v for v in allowed)))
    return False


def validate_args(mode, input_path, out_dir, style, group_mode, video_reader, det_model, enc_model,
                  decoupled=False):
    """prep.py:18-45.  decoupled=True lifts the style <-> model coupling (prep.py:39-44) so that
    e.g. YOLO detection + ViT-L encoding (BASELINE config 5) can be requested explicitly."""
    if not _one_of(mode, 'mode', ['full', 'detection', 'grouping']):
        return False
    ok = True
    if input_path is not None and not isinstance(input_path, str):
        pass  # in-memory frames
    elif input_path and not osp.exists(input_path):
        print("ERROR: specified input_path doesn't exist. Please provide a valid path to a file, a directory "
              "with files, or a .txt file with full paths inside")
        ok = False
    if out_dir and not osp.isdir(out_dir):
        print("ERROR: specified out_dir doesn't exist or isn't a directory. Please provide a valid path to a "
              "directory")
        ok = False
    if input_path is None and mode != 'grouping':
        print('ERROR: please specify input_path')
        ok = False
    if input_path is None and mode == 'grouping' and not out_dir:
        print('ERROR: for grouping, please specify either out_dir or the same input_path used during detection')
        ok = False
    ok = ok and _one_of(style, 'style', ['live', 'anime'])
    ok = ok and _one_of(group_mode, 'group_mode', ['clustering', 'classification'])
    ok = ok and _one_of(video_reader, 'video_reader', ['opencv', 'decord'])
    if decoupled:
        ok = ok and _one_of(det_model, 'det_model', list(dict.fromkeys(LIVE_DET + ANIME_DET)))
        ok = ok and _one_of(enc_model, 'enc_model', list(dict.fromkeys(LIVE_ENC + ANIME_ENC)))
    elif style == 'live':
        ok = ok and _one_of(det_model, 'det_model', LIVE_DET) and _one_of(enc_model, 'enc_model', LIVE_ENC)
    elif style == 'anime':
        ok = ok and _one_of(det_model, 'det_model', ANIME_DET) and _one_of(enc_model, 'enc_model', ANIME_ENC)
    return ok


def get_clusters(c):
    """prep.py:48-66: None -> 2..8, an int, 'a,b,c' or 'a-b'."""
    if not c:
        return list(range(2, 9))
    if isinstance(c, int) and c > 0:
        return [c]
    if isinstance(c, str) and ',' in c:
        parts = c.split(',')
        if all(p.isdigit() for p in parts):
            return sorted(set(int(p) for p in parts))
    if isinstance(c, str):
        parts = c.split('-')
        if len(parts) == 2 and all(p.isdigit() for p in parts):
            a, b = int(parts[0]), int(parts[1])
            if 0 < a < b:
                return list(range(a, b + 1))
    print('ERROR: incorrent value for clusters. Please specify a natural number or a string either as an '
          'enumeration "C1,C2,C3,C4" or a range "A-B" where 0 < A < B')
    return None


def get_class_ref(ref_dir, out_dir):
    """prep.py:69-105: [(class, [image paths])] from the ref_dir subfolders."""
    why = ('Please prepare a directory with 1 or more subfolders representing groups, each with 1 or more '
           'reference images inside')
    if not ref_dir:
        cand = osp.join(out_dir, 'ref')
        if not osp.isdir(cand):
            print('ERROR: for group_mode="classification", ref_dir needs to be specified')
            print(why)
            return None
        print('NOTE: ref_dir is unspecified, but found "ref" folder inside out_dir. Will search for reference '
              'images there')
        ref_dir = cand
    if not osp.isdir(ref_dir):
        print("ERROR: specified ref_dir doesn't exist or isn't a directory. Please provide a valid path to a "
              "directory")
        return None
    classes = sorted(e.name for e in os.scandir(ref_dir) if e.is_dir())
    if not classes:
        print("ERROR: specified ref_dir doesn't contain any subfolders")
        print(why)
        return None
    refs, warns = [], []
    for c in classes:
        imgs = get_img_paths(osp.join(ref_dir, c))
        if imgs:
            refs.append((c, imgs))
        else:
            warns.append('WARNING: ref_dir\'s subfolder "%s" doesn\'t contain any images. During classification, '
                         'this class will be ignored' % c)
    if not refs:
        print("ERROR: none of the ref_dir's subfolders contain any images")
        print('Supported extensions are: %s' % ', '.join(IMG_EXTENSIONS))
        return None
    for w in warns:
        print(w)
    return refs


def get_paths_for_grouping(out_dir):
    """prep.py:108-120: faces/ first, then out_dir itself."""
    for d in (osp.join(out_dir, 'faces'), out_dir):
        paths = get_img_paths(d)
        if paths:
            print('Found %u images at: %s' % (len(paths), d))
            return paths
    print('ERROR: no image files for grouping found at: %s' % out_dir)
    return None


def get_video_list(inp, ext):
    """prep.py:123-146: a .txt list of paths, a single file, or a directory's files."""
    if osp.isfile(inp) and inp.lower().endswith('.txt'):
        with open(inp) as f:
            files = [ln.strip() for ln in f.read().splitlines() if osp.isfile(ln.strip())]
        if not files:
            print("ERROR: specified .txt file doesn't contain any valid paths. Please provide a file with paths to "
                  "videos, each on a separate line")
        return files
    if osp.isfile(inp):
        return [inp]
    files = [osp.join(inp, p) for p in sorted(os.listdir(inp)) if osp.isfile(osp.join(inp, p))]
    if not files:
        print('ERROR: no files are found in the specified input directory')
    if ext:
        files = [f for f in files if f.lower().split('.')[-1] in ext.split(';')]
        if not files:
            print('ERROR: no files with specified extensions (%s) are found in the input directory' % ext)
    return files
